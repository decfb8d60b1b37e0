"""Arch B — classification service: gRPC ``inference.ClassificationService`` on :8201.

Reference: architectures/microservices/classification/app/main.py:29-105
(``grpc.aio`` server, 50 MB message limits, SIGTERM/SIGINT with a 5 s grace)
and servicer.py:45-159 (``Classify`` decodes the crop, runs MobileNetV2,
returns softmax top-1 + top-5 with ``TimingInfo``; failures are reported
in-band in ``error``; ``ClassifyBatch`` loops over ``Classify``).

MI355X design: every RPC only decodes (thread pool) and enqueues its crop
into the GPU classifier's dynamic batcher, so crops of concurrent requests —
and all crops of one ``ClassifyBatch`` — run as one batched MobileNetV2 graph
replay.  ``Health/Check`` is implemented (declared only upstream), and with
``ARENA_INFER_SERVICE=1`` so is ``InferenceService/Infer`` (also declared
only upstream; see server/inference_service.py).  With
``ARENA_CROP_TRANSPORT=device`` requests may name a frame in the detection
process's device memory instead of carrying crop bytes
(server/device_transport.py): those crops are cut and classified on the GPU
straight from the IPC-mapped frame.

Run: ``python -m inference_arena_amd.server.classification_service``.
"""
from __future__ import annotations

import asyncio
import logging
import signal
import time
from concurrent.futures import ThreadPoolExecutor

import grpc

from ..labels import load_labels
from ..proto import inference_api as pb
from ..utils.logging import request_id_var, setup_logging
from ..utils.settings import Settings
from .crop_codec import RAW_MAGIC, decode_crop
from .service_backends import ClassifierBackend, build_classifier_backend

log = logging.getLogger("arena.classification")

MAX_MESSAGE = 50 * 1024 * 1024
GRPC_OPTIONS = [("grpc.max_send_message_length", MAX_MESSAGE), ("grpc.max_receive_message_length", MAX_MESSAGE)]


class ClassificationServicer:
    def __init__(self, backend: ClassifierBackend, labels: list[str], decode_threads: int = 8):
        self.backend = backend
        self.labels = labels
        self.pool = ThreadPoolExecutor(max_workers=max(1, decode_threads), thread_name_prefix="crop-decode")
        self.n_requests = 0
        self.n_errors = 0
        self.infer = None  # InferenceServicer when the server also serves InferenceService
        self.frames = None  # device_transport.DeviceClassifier when device-resident frames are accepted

    def _name(self, cid: int) -> str:
        return self.labels[cid] if 0 <= cid < len(self.labels) else ""

    def _response(self, rid: str, ids, probs, t0: float, t1: float, t2: float):
        top = [pb.ClassificationResult(class_id=c, class_name=self._name(c), confidence=p)
               for c, p in zip(ids, probs)]
        t3 = time.perf_counter()
        return pb.ClassificationResponse(
            request_id=rid, result=top[0], top_k=top,
            timing=pb.TimingInfo(preprocessing_ms=(t1 - t0) * 1e3, inference_ms=(t2 - t1) * 1e3,
                                 postprocessing_ms=(t3 - t2) * 1e3, total_ms=(t3 - t0) * 1e3))

    async def _classify_frames(self, requests) -> list:
        """Crops named by device-resident frames: one DeviceClassifier entry per frame (its crops share it)."""
        from .device_transport import group_by_image

        t0 = time.perf_counter()
        out = [None] * len(requests)
        if self.frames is None:
            for i, r in enumerate(requests):
                out[i] = pb.ClassificationResponse(request_id=r.request_id,
                                                   error="device crop transport not enabled on this service")
            self.n_errors += len(requests)
            return out
        groups = group_by_image(requests)
        t1 = time.perf_counter()
        results = await asyncio.gather(*(self.frames.classify(k, b) for k, b, _ in groups), return_exceptions=True)
        t2 = time.perf_counter()
        for (_, _, idx), res in zip(groups, results):
            for j, i in enumerate(idx):
                rid = requests[i].request_id
                if isinstance(res, BaseException):
                    self.n_errors += 1
                    out[i] = pb.ClassificationResponse(request_id=rid, error=str(res))
                else:
                    out[i] = self._response(rid, res[j][0], res[j][1], t0, t1, t2)
        return out

    async def Classify(self, request, context=None):
        t0 = time.perf_counter()
        request_id_var.set(request.request_id)
        self.n_requests += 1
        if request.HasField("device_image"):
            return (await self._classify_frames([request]))[0]
        try:
            data = request.image_crop
            if data[:4] == RAW_MAGIC:  # raw crops are a header + a view: no codec, no thread hop
                crop = decode_crop(data)
            else:
                crop = await asyncio.get_running_loop().run_in_executor(self.pool, decode_crop, data)
            t1 = time.perf_counter()
            idx, _logit, prob = await self.backend.classify(crop)
            t2 = time.perf_counter()
            return self._response(request.request_id, idx.tolist(), prob.tolist(), t0, t1, t2)
        except Exception as e:  # in-band error, like the reference
            self.n_errors += 1
            log.error(f"Classification failed: {e}")
            return pb.ClassificationResponse(request_id=request.request_id, error=str(e))

    async def ClassifyBatch(self, request, context=None):
        t0 = time.perf_counter()
        reqs = list(request.requests)
        dev = [i for i, r in enumerate(reqs) if r.HasField("device_image")]
        if not dev:
            responses = list(await asyncio.gather(*(self.Classify(r, context) for r in reqs)))
        else:
            self.n_requests += len(dev)
            host = [i for i in range(len(reqs)) if i not in set(dev)]
            dres, hres = await asyncio.gather(self._classify_frames([reqs[i] for i in dev]),
                                              asyncio.gather(*(self.Classify(reqs[i], context) for i in host)))
            responses = [None] * len(reqs)
            for i, r in zip(dev, dres):
                responses[i] = r
            for i, r in zip(host, hres):
                responses[i] = r
        out = pb.BatchClassificationResponse(responses=responses)
        out.batch_timing.total_ms = (time.perf_counter() - t0) * 1e3
        return out

    def close(self) -> None:
        self.pool.shutdown(wait=False)
        if self.frames is not None:
            self.frames.close()
        if self.infer is not None:
            self.infer.backend.close()
            self.infer.close()


class HealthServicer:
    def __init__(self, ready=lambda: True):
        self.ready = ready

    async def Check(self, request, context=None):
        return pb.HealthCheckResponse(status=pb.SERVING if self.ready() else pb.NOT_SERVING)


async def start_server(settings: Settings, backend: ClassifierBackend | None = None, port: int | None = None,
                       pipeline_backend=None, frames=None):
    """Create and start the aio server; returns (server, servicer, bound_port).

    With ``pipeline_backend`` (or ``ARENA_INFER_SERVICE=1``, which builds one) the same
    server also answers ``inference.InferenceService/Infer`` (server/inference_service.py)."""
    backend = backend or build_classifier_backend(settings)
    labels = load_labels(settings.LABELS_FILE or None)
    servicer = ClassificationServicer(backend, labels, settings.ARENA_DECODE_THREADS)
    if frames is None and settings.ARENA_CROP_TRANSPORT == "device" and settings.ARENA_DEVICE != "cpu":
        from .service_backends import build_frame_classifier

        frames = build_frame_classifier(settings)
    servicer.frames = frames
    handlers = [pb.ClassificationService.handler(servicer), pb.Health.handler(HealthServicer())]
    if pipeline_backend is None and int(settings.ARENA_INFER_SERVICE):
        from .inference_service import build_pipeline_backend

        pipeline_backend = build_pipeline_backend(settings)
    if pipeline_backend is not None:
        from .inference_service import InferenceServicer

        servicer.infer = InferenceServicer(pipeline_backend, labels, settings.ARENA_DECODE_THREADS)
        handlers.append(pb.InferenceService.handler(servicer.infer))
    server = grpc.aio.server(options=GRPC_OPTIONS)
    server.add_generic_rpc_handlers(tuple(handlers))
    bound = server.add_insecure_port(f"{settings.HOST}:{port if port is not None else settings.PORT}")
    await server.start()
    log.info("classification service listening", extra={"port": bound})
    return server, servicer, bound


async def serve(settings: Settings) -> None:
    setup_logging(settings.LOG_LEVEL)
    server, servicer, _ = await start_server(settings)
    stop = asyncio.Event()
    loop = asyncio.get_running_loop()
    for sig in (signal.SIGTERM, signal.SIGINT):
        loop.add_signal_handler(sig, stop.set)
    await stop.wait()
    log.info("shutting down classification service (5 s grace)")
    await server.stop(grace=5)
    servicer.backend.close()
    servicer.close()


def main() -> None:
    import os

    s = Settings.from_env()
    if "PORT" not in os.environ:
        s.PORT = 8201
    asyncio.run(serve(s))


if __name__ == "__main__":
    main()
