"""Inference backends shared by every serving topology.

``GpuBatchedBackend``  the MI355X path: requests (decoded RGB) go into the
                       native DynamicBatcher (csrc/runtime/batcher.cpp) over
                       one or more Executor instances; completion callbacks
                       resolve asyncio futures, so the event loop never blocks
                       (the reference's ``async def predict`` calls blocking
                       ONNX Runtime inline and serialises every request,
                       architectures/monolithic/app/main.py:102-159).
``CpuReferenceBackend`` the reference-equivalent CPU arm (BASELINE config 1):
                       the fp32 torch oracles with the upstream 2 intra-op
                       threads, one request at a time.

Both return ``ImageResult`` + a timing dict with the reference's keys
(detection_ms, classification_ms, total_ms) plus queue_ms / gpu_ms /
batch_size.
"""
from __future__ import annotations

import asyncio
import threading
import os
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from ..engine.pipeline import ImageResult
from .batching import AsyncBatcher, Overloaded  # noqa: F401  (re-exported)


class Backend:
    name = "backend"

    def ready(self) -> bool:
        return True

    async def infer(self, image: np.ndarray) -> tuple[ImageResult, dict]:
        raise NotImplementedError

    def stats(self) -> dict:
        return {}

    def close(self) -> None:
        pass


def _result_from_dict(d: dict) -> ImageResult:
    det = d["det"]
    return ImageResult(
        boxes=det[:, :4].copy(),
        scores=det[:, 4].copy(),
        classes=det[:, 5].copy().view(np.int32),
        topk_idx=d["topk_idx"],
        topk_logit=d["topk_logit"],
        topk_prob=d["topk_prob"],
        det_count=int(d["det_count"]),
    )


def settings_devices(settings) -> list[int]:
    """GPUs one service process drives: ``ARENA_GPUS`` ("0,1" / "0-3"), else ``ARENA_GPU``."""
    from ..parallel.placement import parse_gpu_list

    return parse_gpu_list(getattr(settings, "ARENA_GPUS", "") or "", default=int(settings.ARENA_GPU))


class GpuBatchedBackend(Backend):
    name = "gpu"

    def __init__(self, yolo, mnet, *, device: int = 0, instances: int = 1, max_batch: int = 32,
                 preferred: list[int] | None = None, max_queue_delay_us: int = 500, max_queue_size: int = 4096,
                 buckets: list[int] | None = None, weights: np.ndarray | None = None,
                 devices: list[int] | None = None, overlap: int | None = None,
                 idle_queue_delay_us: int | None = None):
        """``instances`` pipelines on each GPU of ``devices`` (default: ``[device]``) behind one batcher queue:
        each instance thread pulls the next batch for its own GPU (data parallel within one process)."""
        from ..engine.registry import build_session

        bk = buckets or sorted({b for b in (1, 2, 4, 8, 16, 32, max_batch) if b <= max_batch})
        self.devices = [int(d) for d in (devices or [device])]
        self.pipes = [build_session("pipeline", yolo, mnet, device=d, buckets=bk, weights=weights)
                      for d in self.devices for _ in range(instances)]
        # overlap (None: ARENA_BATCH_OVERLAP, default on): batches overlap in the free slots — right for one
        # process per GPU (the monolithic arm, native_front.py); the model server's ensemble passes 0 (three
        # processes per GPU: profiles/r5_serving/README.md)
        if overlap is None:
            overlap = int(os.environ.get("ARENA_BATCH_OVERLAP", "1"))
        if idle_queue_delay_us is None:
            idle_queue_delay_us = int(os.environ.get("ARENA_IDLE_QUEUE_DELAY_US", "100"))
        self.batcher = AsyncBatcher(self.pipes, max_batch=max_batch, preferred=preferred,
                                    max_queue_delay_us=max_queue_delay_us, max_queue_size=max_queue_size,
                                    overlap=int(overlap), idle_queue_delay_us=int(idle_queue_delay_us))
        self.device = device

    def ready(self) -> bool:
        return self.batcher.healthy

    @property
    def device_error(self) -> str | None:
        return self.batcher.device_error

    async def infer(self, image: np.ndarray) -> tuple[ImageResult, dict]:
        t0 = time.perf_counter()
        d = await self.batcher.run(np.ascontiguousarray(image, dtype=np.uint8))
        return self._finish(d, t0)

    async def infer_bytes(self, data: bytes, decode) -> tuple[ImageResult, dict]:
        """An encoded upload through the native split decoder (batching.AsyncBatcher.run_jpeg); ``decode`` is
        the fallback for formats it does not cover."""
        t0 = time.perf_counter()
        d = await self.batcher.run_jpeg(data, decode, threads=int(os.environ.get("ARENA_INGEST_THREADS", "4")))
        return self._finish(d, t0)

    def _finish(self, d: dict, t0: float) -> tuple[ImageResult, dict]:
        total = (time.perf_counter() - t0) * 1e3
        q = d["queue_us"] / 1e3
        gpu = d["compute_us"] / 1e3
        # device time of the two networks in this request's batch (the program's wall-clock stamps, executor
        # OP_STAMP); together with H2D / D2H they make up gpu_ms.  Programs without stamps report 0.
        det_ms, cls_ms = float(d.get("detection_ms", -1.0)), float(d.get("classification_ms", -1.0))
        timing = {"queue_ms": q, "gpu_ms": gpu, "batch_size": float(d["batch_size"]),
                  "detection_ms": max(0.0, det_ms), "classification_ms": max(0.0, cls_ms), "inference_ms": total}
        return _result_from_dict(d), timing

    def stats(self) -> dict:
        return self.batcher.stats()

    def close(self) -> None:
        self.batcher.close()


def fake_instance(max_batch: int = 8):
    """Host-only stand-in for one device (``ARENA_DEVICE=fake``, CPU tests of the node layouts): the native
    EchoInstance answers every batch after ``ARENA_FAKE_LATENCY_US`` (default 20 ms) with ``ARENA_FAKE_SLOTS``
    (default 2) batches in flight, so one fake device serves at most slots x max_batch / latency requests/s
    whatever the host does; N ranks scale only if their host layout does."""
    from ..ops import native

    mb = int(os.environ.get("ARENA_FAKE_MAX_BATCH", "0") or 0) or int(max_batch)
    return native().EchoInstance(int(os.environ.get("ARENA_FAKE_SLOTS", "2")), mb, 4,
                                 int(os.environ.get("ARENA_FAKE_LATENCY_US", "20000")))


class FakeBatchedBackend(GpuBatchedBackend):
    """The GPU backend's interface (native DynamicBatcher, ``infer`` / ``infer_bytes``) over ``fake_instance``."""

    name = "fake"

    def __init__(self, *, max_batch: int = 8, max_queue_delay_us: int = 500, overlap: int = 1):
        class _Inst:
            def __init__(self, ex):
                self.ex = ex

        max_batch = int(os.environ.get("ARENA_FAKE_MAX_BATCH", "0") or 0) or int(max_batch)
        self.devices = [0]
        self.pipes = [_Inst(fake_instance(max_batch))]
        self.batcher = AsyncBatcher(self.pipes, max_batch=max_batch, max_queue_delay_us=max_queue_delay_us,
                                    overlap=int(overlap))
        self.device = 0


class GpuSplitBackend(GpuBatchedBackend):
    """Monolithic arm in the split topology: detection on ``det_device``, classification on ``cls_device``
    (engine.pipeline.SplitPipeline: crop plan, detections and images handed over device to device) behind
    the native dynamic batcher."""

    def __init__(self, yolo, mnet, *, det_device: int = 0, cls_device: int = 1, instances: int = 1,
                 max_batch: int = 32, preferred: list[int] | None = None, max_queue_delay_us: int = 500,
                 max_queue_size: int = 4096, buckets: list[int] | None = None):
        from ..engine.registry import build_session

        bk = buckets or sorted({b for b in (1, 2, 4, 8, 16, 32, max_batch) if b <= max_batch})
        self.devices = [int(det_device), int(cls_device)]
        self.pipes = [build_session("split", yolo, mnet, device=det_device, cls_device=cls_device, buckets=bk)
                      for _ in range(instances)]

        class _Inst:  # AsyncBatcher schedules `.ex`: the split batch instance
            def __init__(self, p):
                self.ex = p.instance

        self.batcher = AsyncBatcher([_Inst(p) for p in self.pipes], max_batch=max_batch, preferred=preferred,
                                    max_queue_delay_us=max_queue_delay_us, max_queue_size=max_queue_size)
        self.device = det_device


class CpuReferenceBackend(Backend):
    name = "cpu"

    def __init__(self, yolo, mnet, *, threads: int = 2, conf_thr: float = 0.5, iou_thr: float = 0.45):
        import torch

        from ..engine.reference import ReferencePipeline

        torch.set_num_threads(threads)
        self.ref = ReferencePipeline(yolo, mnet, conf_thr=conf_thr, iou_thr=iou_thr, device="cpu")
        # one worker: the reference processes requests one at a time
        self.pool = ThreadPoolExecutor(max_workers=1, thread_name_prefix="cpu-infer")
        self.lock = threading.Lock()

    def _run(self, image: np.ndarray):
        from ..processing import extract_crop

        with self.lock:
            t0 = time.perf_counter()
            det = self.ref.detect(image)
            t1 = time.perf_counter()
            logits = self.ref.classify([extract_crop(image, d) for d in det])
            t2 = time.perf_counter()
        k = len(det)
        order = np.argsort(-logits, axis=1, kind="stable")[:, :5] if k else np.zeros((0, 5), np.int64)
        top = np.take_along_axis(logits, order, 1) if k else np.zeros((0, 5), np.float32)
        if k:
            z = np.exp(logits - logits.max(1, keepdims=True))
            prob = np.take_along_axis(z / z.sum(1, keepdims=True), order, 1)
        else:
            prob = np.zeros((0, 5), np.float32)
        res = ImageResult(boxes=det[:, :4].astype(np.float32) if k else np.zeros((0, 4), np.float32),
                          scores=det[:, 4].astype(np.float32) if k else np.zeros((0,), np.float32),
                          classes=det[:, 5].astype(np.int32) if k else np.zeros((0,), np.int32),
                          topk_idx=order.astype(np.int32), topk_logit=top.astype(np.float32),
                          topk_prob=prob.astype(np.float32), det_count=k)
        return res, {"detection_ms": (t1 - t0) * 1e3, "classification_ms": (t2 - t1) * 1e3}

    async def infer(self, image: np.ndarray) -> tuple[ImageResult, dict]:
        loop = asyncio.get_running_loop()
        return await loop.run_in_executor(self.pool, self._run, image)

    def close(self) -> None:
        self.pool.shutdown(wait=False)


def build_backend(settings, *, arch: str = "monolithic") -> Backend:
    """Backend selected by ARENA_DEVICE (gpu | cpu) with the arena's default models."""
    from ..config import get_triton_config
    from ..models.zoo import resolve_models

    yolo, mnet = resolve_models(settings.MODELS_DIR, int(settings.ARENA_WEIGHT_SEED))
    if settings.ARENA_DEVICE == "cpu":
        from ..config import get_controlled_variable

        return CpuReferenceBackend(yolo, mnet, threads=int(get_controlled_variable("onnx_runtime",
                                                                                     "intra_op_num_threads")))
    db = get_triton_config().get("dynamic_batching", {}) or {}
    if int(getattr(settings, "ARENA_CLS_GPU", -1)) >= 0:  # split topology: classification on another GPU
        return GpuSplitBackend(yolo, mnet, det_device=int(settings.ARENA_GPU), cls_device=int(settings.ARENA_CLS_GPU),
                               max_batch=int(settings.ARENA_MAX_BATCH),
                               preferred=list(db.get("preferred_batch_size", [])),
                               max_queue_delay_us=int(settings.ARENA_QUEUE_DELAY_US))
    return GpuBatchedBackend(yolo, mnet, device=int(settings.ARENA_GPU), devices=settings_devices(settings),
                             max_batch=int(settings.ARENA_MAX_BATCH),
                             preferred=list(db.get("preferred_batch_size", [])),
                             max_queue_delay_us=int(settings.ARENA_QUEUE_DELAY_US))
