"""``inference.InferenceService/Infer`` — the whole pipeline as one gRPC call.

The reference declares this service (src/shared/proto/inference.proto:137-152:
``InferenceRequest{request_id, image, detection_threshold, max_detections,
top_k}`` -> ``InferenceResponse{request_id, results[], timing, error}``) but
never implements it.  Here it is served over the same fused GPU pipeline
backend as the monolithic ``/predict`` (``server/backends.py``): the encoded
image is decoded on a thread pool, enqueued into the native dynamic batcher,
and the detections + classifications come back in one response.

Semantics (documented choices where the proto leaves them open):
  * ``detection_threshold`` > 0 filters detections *above* the pipeline's
    own threshold (the device program is compiled at experiment.yaml's 0.5,
    so a lower request threshold cannot add detections);
  * ``max_detections`` > 0 keeps the highest-scoring detections only;
  * ``top_k`` is accepted for wire compatibility; the result carries top-1
    (the message has a single ``classification`` per detection);
  * classification ``confidence`` is the softmax probability (arm B's
    convention) unless the servicer is built with ``confidence="logit"``;
  * failures are reported in-band in ``error`` (the reference's gRPC style,
    architectures/microservices/classification/app/servicer.py:121-126).

Served by ``python -m inference_arena_amd.server.classification_service``
when ``ARENA_INFER_SERVICE=1`` (on the classification port), or standalone:
``python -m inference_arena_amd.server.inference_service`` (:8202).
"""
from __future__ import annotations

import asyncio
import logging
import signal
import time

import grpc
import numpy as np

from ..labels import load_labels
from ..proto import inference_api as pb
from ..utils.logging import request_id_var, setup_logging
from ..utils.settings import Settings
from .app_common import DecodePool
from .backends import Backend

log = logging.getLogger("arena.inference_service")

MAX_MESSAGE = 50 * 1024 * 1024
GRPC_OPTIONS = [("grpc.max_send_message_length", MAX_MESSAGE), ("grpc.max_receive_message_length", MAX_MESSAGE)]


def select_detections(scores: np.ndarray, threshold: float, max_detections: int) -> np.ndarray:
    """Indices of the detections an ``InferenceRequest`` keeps, in pipeline order
    (class id asc, score desc) — threshold first, then the top ``max_detections`` by score."""
    keep = np.arange(len(scores))
    if threshold > 0:
        keep = keep[scores[keep] >= threshold]
    if max_detections > 0 and len(keep) > max_detections:
        best = np.argsort(-scores[keep], kind="stable")[:max_detections]
        keep = np.sort(keep[best])
    return keep


class InferenceServicer:
    def __init__(self, backend: Backend, labels: list[str], decode_threads: int = 8, confidence: str = "softmax"):
        if confidence not in ("softmax", "logit"):
            raise ValueError("confidence must be 'softmax' or 'logit'")
        self.backend = backend
        self.labels = labels
        self.confidence = confidence
        self.decoder = DecodePool(decode_threads)
        self.n_requests = 0
        self.n_errors = 0

    def _name(self, cid: int) -> str:
        return self.labels[cid] if 0 <= cid < len(self.labels) else ""

    async def Infer(self, request, context=None):
        t0 = time.perf_counter()
        request_id_var.set(request.request_id)
        self.n_requests += 1
        try:
            if not request.image:
                raise ValueError("empty image")
            image = await self.decoder.decode(request.image)
            t1 = time.perf_counter()
            res, _timing = await self.backend.infer(image)
            t2 = time.perf_counter()
            resp = pb.InferenceResponse(request_id=request.request_id)
            keep = select_detections(res.scores, float(request.detection_threshold), int(request.max_detections))
            for i in keep:
                r = resp.results.add()
                x1, y1, x2, y2 = (float(v) for v in res.boxes[i])
                r.detection.x1, r.detection.y1, r.detection.x2, r.detection.y2 = x1, y1, x2, y2
                r.detection.confidence = float(res.scores[i])
                r.detection.class_id = int(res.classes[i])
                if i < len(res.topk_idx):
                    cid = int(res.topk_idx[i][0])
                    r.classification.class_id = cid
                    r.classification.class_name = self._name(cid)
                    src = res.topk_prob if self.confidence == "softmax" else res.topk_logit
                    r.classification.confidence = float(src[i][0])
            t3 = time.perf_counter()
            resp.timing.preprocessing_ms = (t1 - t0) * 1e3
            resp.timing.inference_ms = (t2 - t1) * 1e3
            resp.timing.postprocessing_ms = (t3 - t2) * 1e3
            resp.timing.total_ms = (t3 - t0) * 1e3
            return resp
        except Exception as e:  # in-band error
            self.n_errors += 1
            log.error(f"Inference failed: {e}")
            return pb.InferenceResponse(request_id=request.request_id, error=str(e))

    def close(self) -> None:
        self.decoder.close()


def build_pipeline_backend(settings: Settings) -> Backend:
    from .backends import build_backend

    return build_backend(settings, arch="inference_service")


async def start_server(settings: Settings, backend: Backend | None = None, port: int | None = None):
    """Standalone InferenceService (+ Health) server; returns (server, servicer, bound_port)."""
    from .classification_service import HealthServicer

    backend = backend or build_pipeline_backend(settings)
    servicer = InferenceServicer(backend, load_labels(settings.LABELS_FILE or None), settings.ARENA_DECODE_THREADS)
    server = grpc.aio.server(options=GRPC_OPTIONS)
    server.add_generic_rpc_handlers((pb.InferenceService.handler(servicer),
                                     pb.Health.handler(HealthServicer(backend.ready))))
    bound = server.add_insecure_port(f"{settings.HOST}:{port if port is not None else settings.PORT}")
    await server.start()
    log.info("inference service listening", extra={"port": bound})
    return server, servicer, bound


async def serve(settings: Settings) -> None:
    setup_logging(settings.LOG_LEVEL)
    server, servicer, _ = await start_server(settings)
    stop = asyncio.Event()
    loop = asyncio.get_running_loop()
    for sig in (signal.SIGTERM, signal.SIGINT):
        loop.add_signal_handler(sig, stop.set)
    await stop.wait()
    await server.stop(grace=5)
    servicer.backend.close()
    servicer.close()


def main() -> None:
    import os

    s = Settings.from_env()
    if "PORT" not in os.environ:
        s.PORT = 8202
    asyncio.run(serve(s))


if __name__ == "__main__":
    main()
