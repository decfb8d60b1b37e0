"""Split-stage backends for the microservices arm (detection :8200,
classification :8201) and their CPU reference equivalents.

GPU: each stage is its own executor program behind the native dynamic
batcher — ``GpuDetector`` (letterbox -> YOLO -> decode -> NMS) and
``GpuClassifier`` (resize/normalise -> MobileNetV2 -> softmax top-5) — so
concurrent ``Classify`` RPCs from many requests are micro-batched on the
device instead of being run one by one inside the async handler as in the
reference (architectures/microservices/classification/app/servicer.py:82).

CPU: fp32 torch oracles with the reference's two intra-op threads
(experiment.yaml onnx_runtime section), one call at a time.
"""
from __future__ import annotations

import asyncio
import os
import threading
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from .batching import AsyncBatcher


def _default_buckets(max_batch: int) -> list[int]:
    return sorted({b for b in (1, 2, 4, 8, 16, 32, 64, max_batch) if b <= max_batch})


class ClassifierBackend:
    """``await classify(crop) -> (top5 ids, top5 logits, top5 softmax probs)``."""

    name = "classifier"

    async def classify(self, crop: np.ndarray):
        raise NotImplementedError

    async def classify_many(self, crops: list[np.ndarray]):
        return list(await asyncio.gather(*(self.classify(c) for c in crops)))

    def stats(self) -> dict:
        return {}

    def close(self) -> None:
        pass


class GpuClassifierBackend(ClassifierBackend):
    name = "gpu"

    def __init__(self, mnet, *, device: int = 0, instances: int = 1, max_batch: int = 64,
                 max_queue_delay_us: int = 300, preferred: list[int] | None = None,
                 devices: list[int] | None = None, idle_queue_delay_us: int = -1):
        from ..engine.registry import build_session

        bk = _default_buckets(max_batch)
        self.devices = [int(d) for d in (devices or [device])]
        self.runners = [build_session("classifier", mnet=mnet, device=d, buckets=bk)
                        for d in self.devices for _ in range(instances)]
        self.batcher = AsyncBatcher(self.runners, max_batch=max_batch, preferred=preferred,
                                    max_queue_delay_us=max_queue_delay_us, idle_queue_delay_us=idle_queue_delay_us)

    def ready(self) -> bool:
        return self.batcher.healthy

    @property
    def device_error(self) -> str | None:
        return self.batcher.device_error

    async def classify(self, crop: np.ndarray):
        d = await self.batcher.run(np.ascontiguousarray(crop, dtype=np.uint8))
        return d["topk_idx"][0], d["topk_logit"][0], d["topk_prob"][0]

    def stats(self) -> dict:
        return self.batcher.stats()

    def close(self) -> None:
        self.batcher.close()


class CpuClassifierBackend(ClassifierBackend):
    name = "cpu"

    def __init__(self, mnet, *, threads: int = 2):
        import copy

        import torch

        from ..processing import MobileNetPreprocessor

        torch.set_num_threads(threads)
        self.mnet = copy.deepcopy(mnet).cpu().eval()
        self.pre = MobileNetPreprocessor()
        self.pool = ThreadPoolExecutor(max_workers=1, thread_name_prefix="cls-cpu")

    def _run(self, crop: np.ndarray):
        import torch

        with torch.no_grad():
            logits = self.mnet(torch.from_numpy(self.pre(crop).tensor)).numpy()[0]
        order = np.argsort(-logits, kind="stable")[:5]
        z = np.exp(logits - logits.max())
        prob = z / z.sum()
        return order.astype(np.int32), logits[order].astype(np.float32), prob[order].astype(np.float32)

    async def classify(self, crop: np.ndarray):
        return await asyncio.get_running_loop().run_in_executor(self.pool, self._run, crop)

    def close(self) -> None:
        self.pool.shutdown(wait=False)


class DetectorBackend:
    """``await detect(image) -> (det [K,6] x1,y1,x2,y2,conf,cls in original coords, timing)``."""

    name = "detector"

    async def detect(self, image: np.ndarray):
        raise NotImplementedError

    def stats(self) -> dict:
        return {}

    def close(self) -> None:
        pass


class GpuDetectorBackend(DetectorBackend):
    name = "gpu"

    def __init__(self, yolo, *, device: int = 0, instances: int = 1, max_batch: int = 32,
                 max_queue_delay_us: int = 500, preferred: list[int] | None = None,
                 devices: list[int] | None = None):
        from ..engine.registry import build_session

        bk = _default_buckets(max_batch)
        self.devices = [int(d) for d in (devices or [device])]
        self.runners = [build_session("detector", yolo, device=d, buckets=bk)
                        for d in self.devices for _ in range(instances)]
        self.batcher = AsyncBatcher(self.runners, max_batch=max_batch, preferred=preferred,
                                    max_queue_delay_us=max_queue_delay_us)

    def ready(self) -> bool:
        return self.batcher.healthy

    @property
    def device_error(self) -> str | None:
        return self.batcher.device_error

    exports_frames = True  # detect(export_to=...) copies the staged frame to a device buffer (arm B device ring)

    async def detect_bytes(self, data: bytes, decode, export_to: int = 0):
        """An encoded upload through the native split decoder (the frame is reconstructed on the GPU inside the
        batch and, with ``export_to``, copied into the device ring from there); ``decode`` is the fallback."""
        d = await self.batcher.run_jpeg(data, decode, threads=int(os.environ.get("ARENA_INGEST_THREADS", "4")),
                                        export_to=export_to)
        return self._detections(d)

    async def detect(self, image: np.ndarray, export_to: int = 0):
        d = await self.batcher.run(np.ascontiguousarray(image, dtype=np.uint8), export_to=export_to)
        return self._detections(d)

    @staticmethod
    def _detections(d: dict):
        det = d["det"]
        out = np.concatenate([det[:, :5], det[:, 5:6].copy().view(np.int32).astype(np.float32)], 1)
        return out, {"queue_ms": d["queue_us"] / 1e3, "gpu_ms": d["compute_us"] / 1e3,
                     "batch_size": float(d["batch_size"])}

    def stats(self) -> dict:
        return self.batcher.stats()

    def close(self) -> None:
        self.batcher.close()


class CpuDetectorBackend(DetectorBackend):
    name = "cpu"

    def __init__(self, yolo, *, threads: int = 2, conf_thr: float = 0.5, iou_thr: float = 0.45):
        import copy

        import torch

        from ..processing import YOLOPreprocessor

        torch.set_num_threads(threads)
        self.yolo = copy.deepcopy(yolo).cpu().eval()
        self.pre = YOLOPreprocessor()
        self.conf_thr, self.iou_thr = conf_thr, iou_thr
        self.pool = ThreadPoolExecutor(max_workers=1, thread_name_prefix="det-cpu")
        self.lock = threading.Lock()

    def _run(self, image: np.ndarray):
        import torch

        from ..postprocess import parse_yolo_output

        t0 = time.perf_counter()
        r = self.pre(image)
        with torch.no_grad():
            out = self.yolo(torch.from_numpy(r.tensor)).numpy()
        det = parse_yolo_output(out, self.conf_thr, self.iou_thr)
        det = r.scale_boxes_to_original(det) if len(det) else np.zeros((0, 6), np.float32)
        return det.astype(np.float32), {"gpu_ms": 0.0, "cpu_ms": (time.perf_counter() - t0) * 1e3}

    async def detect(self, image: np.ndarray):
        return await asyncio.get_running_loop().run_in_executor(self.pool, self._run, image)

    def close(self) -> None:
        self.pool.shutdown(wait=False)


def build_classifier_backend(settings) -> ClassifierBackend:
    from ..config import get_controlled_variable
    from ..models.zoo import resolve_models

    _, mnet = resolve_models(settings.MODELS_DIR, int(settings.ARENA_WEIGHT_SEED))
    if settings.ARENA_DEVICE == "cpu":
        return CpuClassifierBackend(mnet, threads=int(get_controlled_variable("onnx_runtime",
                                                                              "intra_op_num_threads")))
    from .backends import settings_devices

    # one classification batch holds the crops of about one detection batch (reference fan-out mu = 4)
    return GpuClassifierBackend(mnet, device=int(settings.ARENA_GPU), devices=settings_devices(settings),
                                max_batch=int(os.environ.get("ARENA_CLS_MAX_BATCH", "0"))
                                or max(32, 4 * int(settings.ARENA_MAX_BATCH)),
                                # ARENA_CLS_QUEUE_DELAY_US (default 2 ms): the classifier's own delay; with 500 us
                                # its batches stayed at a few crops (2.50k vs 2.86k req/s at 50 users, 2.68k vs 2.94k
                                # at 100; 4 ms cost 27 % at 10 users; profiles/serving_r2d/cls_delay/)
                                max_queue_delay_us=int(os.environ.get("ARENA_CLS_QUEUE_DELAY_US", "2000")),
                                # while no batch is in flight the detection side's short delay applies, so a lone
                                # request is not held for 2 ms (1 user: P50 6.8 ms with 2 ms, 5.1 ms with 0.5 ms)
                                idle_queue_delay_us=int(settings.ARENA_QUEUE_DELAY_US))


def build_frame_classifier(settings):
    """Classification side of ``ARENA_CROP_TRANSPORT=device``: a ``GpuFrameClassifier`` (crop gather +
    MobileNetV2 over device-resident frames) behind the frame micro-batcher of server/device_transport.py."""
    from ..engine.registry import build_session
    from ..models.zoo import resolve_models
    from ..ops import native
    from .device_transport import DeviceClassifier

    _, mnet = resolve_models(settings.MODELS_DIR, int(settings.ARENA_WEIGHT_SEED))
    dev = int(settings.ARENA_GPU)
    max_batch = int(settings.ARENA_MAX_BATCH)
    runner = build_session("frame_classifier", mnet=mnet, device=dev, buckets=_default_buckets(max_batch))
    C = native()
    return DeviceClassifier(runner, lambda h: C.ipc_open_range(h, dev), max_batch=max_batch,
                            peer_check=lambda src: C.require_peer_access(dev, src, "device transport"),
                            max_crops=int(runner.ex.crop_cap_for(runner.max_batch)),
                            max_delay_us=int(os.environ.get("ARENA_CLS_QUEUE_DELAY_US", "300")))


def build_detector_backend(settings) -> DetectorBackend:
    from ..config import get_controlled_variable, get_model_config
    from ..models.zoo import resolve_models

    yolo, _ = resolve_models(settings.MODELS_DIR, int(settings.ARENA_WEIGHT_SEED))
    if settings.ARENA_DEVICE == "cpu":
        y = get_model_config("yolov5n")
        return CpuDetectorBackend(yolo, threads=int(get_controlled_variable("onnx_runtime", "intra_op_num_threads")),
                                  conf_thr=float(y["confidence_threshold"]), iou_thr=float(y["iou_threshold"]))
    from .backends import settings_devices

    return GpuDetectorBackend(yolo, device=int(settings.ARENA_GPU), devices=settings_devices(settings),
                              max_batch=int(settings.ARENA_MAX_BATCH),
                              max_queue_delay_us=int(settings.ARENA_QUEUE_DELAY_US))
