"""Arch C — gateway: FastAPI ``POST /predict`` on :8300 in front of the model server.

Reference: architectures/triton/gateway/app/main.py:31-155 and
pipeline.py:102-207 — lifespan waits for the server (backoff) and checks both
models' metadata; ``predict`` letterboxes on the gateway CPU, sends the FP32
tensor to ``yolov5n``, runs NMS on the CPU, then classifies every crop with
a **serial** ``mobilenetv2`` call (confidence = raw logit).

Modes (``ARENA_GATEWAY_MODE``)
  ``pipeline`` (default, MI355X design): the encoded image goes to the
      ``arena_pipeline`` ensemble in ONE RPC; the server runs the fused
      device program (≈100 KB on the wire instead of ≈10 MB per request).
  ``tensor``   the reference protocol, kept for comparison: per-model tensor
      RPCs (crops serial by default; ``ARENA_FANOUT=parallel`` gathers them).
"""
from __future__ import annotations

import asyncio
import logging
from contextlib import asynccontextmanager

import numpy as np
from fastapi import FastAPI, HTTPException, Request
from fastapi.responses import Response

from ..labels import load_labels
from ..metrics import ArenaMetrics
from ..postprocess import parse_yolo_output
from ..processing import MobileNetPreprocessor, YOLOPreprocessor, extract_crop
from ..utils.logging import request_id_var, setup_logging
from ..utils.settings import Settings
from .app_common import DecodePool, FaultInjector, Timer, device_fault, new_request_id, read_upload
from .kserve_client import ModelServerClient
from .schemas import Classification, DetectionBox, DetectionWithClassification, HealthResponse, PredictResponse

log = logging.getLogger("arena.gateway")


def create_app(settings: Settings | None = None, client: ModelServerClient | None = None) -> FastAPI:
    settings = settings or Settings.from_env(PORT=None)
    state: dict = {"client": client, "ready": False}

    @asynccontextmanager
    async def lifespan(app: FastAPI):
        setup_logging(settings.LOG_LEVEL)
        state["labels"] = load_labels(settings.LABELS_FILE or None)
        state["decode"] = DecodePool(settings.ARENA_DECODE_THREADS)
        state["metrics"] = ArenaMetrics("triton", str(settings.ARENA_GPU))
        state["faults"] = FaultInjector(settings.ARENA_FAULT_EVERY)
        state["ypre"], state["mpre"] = YOLOPreprocessor(), MobileNetPreprocessor()
        if state["client"] is None:
            state["client"] = ModelServerClient(settings.TRITON_GRPC_ENDPOINT, settings.TRITON_TIMEOUT_SECONDS)
        cl: ModelServerClient = state["client"]
        if not await cl.wait_for_server_ready(settings.TRITON_TIMEOUT_SECONDS):
            raise RuntimeError(f"model server at {settings.TRITON_GRPC_ENDPOINT} not ready")
        models = ["arena_pipeline"] if settings.ARENA_GATEWAY_MODE == "pipeline" else ["yolov5n", "mobilenetv2"]
        for m in models:
            md = await cl.get_model_metadata(m)
            log.info(f"model {m}: inputs {[t['name'] for t in md['inputs']]}")
        state["ready"] = True
        yield
        await cl.close()
        state["decode"].close()

    app = FastAPI(title="Gateway (MI355X model server)", version="2.0.0", lifespan=lifespan)
    app.state.arena = state

    def _cls(cid: int, conf: float) -> Classification:
        labels = state["labels"]
        return Classification(class_id=cid, class_name=labels[cid] if 0 <= cid < len(labels) else "",
                              confidence=conf)

    def _box(d) -> DetectionBox:
        return DetectionBox(x1=float(d[0]), y1=float(d[1]), x2=float(d[2]), y2=float(d[3]),
                            confidence=float(d[4]), class_id=int(d[5]))

    async def predict_pipeline(rid: str, data: bytes):
        cl: ModelServerClient = state["client"]
        t = Timer()
        out = await cl.infer_pipeline(data, request_id=rid)
        ms = t.ms()
        det = out["DETECTIONS"]
        conf_kind = settings.ARENA_CONFIDENCE or "logit"
        conf = out["CLASS_PROBS"] if conf_kind == "softmax" else out["CLASS_LOGITS"]
        dets = [DetectionWithClassification(detection=_box(det[i]),
                                            classification=_cls(int(out["CLASS_IDS"][i, 0]), float(conf[i, 0])))
                for i in range(det.shape[0])]
        st = out.get("STAGE_MS")
        timing = {"inference_ms": ms}
        if st is not None and np.asarray(st).size >= 4:
            st = np.asarray(st, np.float64).ravel()
            timing.update({"detection_ms": float(st[0]), "classification_ms": float(st[1]),
                           "queue_ms": float(st[2]), "gpu_ms": float(st[3])})
        else:  # a model server without stage outputs: the whole round trip counts as detection
            timing.update({"detection_ms": ms, "classification_ms": 0.0})
        return dets, timing

    async def predict_tensor(rid: str, data: bytes):
        cl: ModelServerClient = state["client"]
        image = await state["decode"].decode(data)
        t = Timer()
        r = state["ypre"](image)
        out = await cl.infer_yolo(r.tensor)
        det = parse_yolo_output(out, 0.5, 0.45)
        det = r.scale_boxes_to_original(det) if len(det) else det
        detection_ms = t.ms()
        t = Timer()

        async def one(d):
            logits = await cl.infer_mobilenet(state["mpre"](extract_crop(image, d)).tensor)
            cid = int(np.argmax(logits[0]))
            return DetectionWithClassification(detection=_box(d), classification=_cls(cid, float(logits[0, cid])))

        if settings.ARENA_FANOUT == "parallel":
            dets = list(await asyncio.gather(*(one(d) for d in det)))
        else:
            dets = [await one(d) for d in det]
        return dets, {"detection_ms": detection_ms, "classification_ms": t.ms()}

    async def predict_bytes(data: bytes) -> PredictResponse:
        """The /predict handler on the upload's bytes (shared by FastAPI and the native front end)."""
        rid = new_request_id()
        tm = Timer()
        metrics: ArenaMetrics = state["metrics"]
        if not state["ready"]:
            metrics.observe("unavailable")
            raise HTTPException(status_code=503, detail="Service not ready")
        try:
            state["faults"].check()
            if settings.ARENA_GATEWAY_MODE == "pipeline":
                dets, timing = await predict_pipeline(rid, data)
            else:
                dets, timing = await predict_tensor(rid, data)
        except Exception as e:
            metrics.observe("error")
            log.error(f"Predict failed: {e}", extra={"endpoint": "/predict", "status_code": 500})
            raise HTTPException(status_code=500, detail=str(e)) from e
        timing["total_ms"] = tm.ms()
        metrics.observe("ok", {k: v for k, v in timing.items() if k.endswith("_ms")}, len(dets), 1)
        log.info("Predict complete", extra={"endpoint": "/predict", "latency_ms": timing["total_ms"],
                                            "detections": len(dets), "status_code": 200})
        return PredictResponse(request_id=rid, detections=dets, timing=timing)

    state["predict_bytes"] = predict_bytes
    state["healthy"] = lambda: bool(state["ready"]) and device_fault(state) is None

    @app.post("/predict", response_model=PredictResponse)
    async def predict(request: Request):
        if not state["ready"]:
            state["metrics"].observe("unavailable")
            raise HTTPException(status_code=503, detail="Service not ready")
        return await predict_bytes(await read_upload(request))

    @app.get("/health", response_model=HealthResponse)
    async def health():
        request_id_var.set(None)
        return HealthResponse(status="healthy", models_loaded=bool(state["ready"]))

    @app.get("/metrics")
    async def metrics_ep():
        return Response(state["metrics"].render(), media_type="text/plain; version=0.0.4")

    return app


def main() -> None:
    import os

    import uvicorn

    s = Settings.from_env()
    if "PORT" not in os.environ:
        s.PORT = 8300
    uvicorn.run(create_app(s), host=s.HOST, port=s.PORT, log_level="warning", access_log=False)


if __name__ == "__main__":
    main()
