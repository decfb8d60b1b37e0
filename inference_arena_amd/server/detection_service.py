"""Arch B — detection service: FastAPI ``POST /predict`` on :8200.

Reference: architectures/microservices/detection/app/main.py:29-121 and
inference.py:99-206 — decode, YOLO in-process, extract every crop, fan the
crops out to the classification service with one ``Classify`` RPC each via
``asyncio.gather``, drop crops whose response carries ``error``, answer with
the shared ``PredictResponse`` (confidence = softmax probability, as the
classification service returns it).

MI355X design: detection is the ``GpuDetector`` program behind the native
dynamic batcher (concurrent requests share one batched YOLO replay); the
event loop never blocks.  ``ARENA_FANOUT=batch`` sends one ``ClassifyBatch``
per request instead of N RPCs; ``ARENA_CROP_TRANSPORT`` picks jpeg (reference)
/ png / raw crops, or ``device``: the decoded frame goes into a ring of IPC-shared
device memory and one ``ClassifyBatch`` names it with the boxes; the
classification service cuts the crops on its GPU (server/device_transport.py).

Run: ``python -m inference_arena_amd.server.detection_service``.
"""
from __future__ import annotations

import asyncio
import logging
import os
from contextlib import asynccontextmanager

from fastapi import FastAPI, HTTPException, Request
from fastapi.responses import JSONResponse, Response

from ..metrics import ArenaMetrics
from ..processing import extract_crop
from ..utils.logging import request_id_var, setup_logging
from ..utils.settings import Settings
from .app_common import DecodePool, FaultInjector, Timer, device_fault, new_request_id, probe_size, read_upload
from .batching import Overloaded
from .grpc_client import ClassificationClient, make_classification_client
from .schemas import Classification, DetectionBox, DetectionWithClassification, HealthResponse, PredictResponse
from .service_backends import DetectorBackend, build_detector_backend

log = logging.getLogger("arena.detection")



async def _detect_holding_slot(coro, ring, slot):
    """Await a detection whose native batch may copy its frame into IPC ring ``slot`` (export_to) and release the
    slot if the detection fails.  A cancelled request (client gone, deadline) must not hand the slot back while
    that batch is still queued or running: its device-to-device export would later overwrite the frame of the
    request that reuses the slot.  The detection is shielded, so it runs to completion, and the slot
    is released from its done-callback."""
    task = asyncio.ensure_future(coro)
    try:
        return await asyncio.shield(task)
    except BaseException:
        if slot is not None:
            if task.done():
                ring.release(slot)
            else:
                def _late(t, s=slot):
                    if not t.cancelled():
                        t.exception()  # retrieved: no "exception was never retrieved" warning
                    ring.release(s)

                task.add_done_callback(_late)
        raise

def create_app(settings: Settings | None = None, detector: DetectorBackend | None = None,
               client: ClassificationClient | None = None, ring=None) -> FastAPI:
    settings = settings or Settings.from_env(PORT=None)
    state: dict = {"detector": detector, "client": client, "ring": ring}

    @asynccontextmanager
    async def lifespan(app: FastAPI):
        setup_logging(settings.LOG_LEVEL)
        log.info("starting detection service", extra={"port": settings.PORT})
        state["decode"] = DecodePool(settings.ARENA_DECODE_THREADS)
        state["metrics"] = ArenaMetrics("microservices", str(settings.ARENA_GPU))
        state["faults"] = FaultInjector(settings.ARENA_FAULT_EVERY)
        if state["detector"] is None:
            state["detector"] = build_detector_backend(settings)
        if state["client"] is None:
            # one endpoint, or a least-outstanding pool over one classification service per GPU
            state["client"] = make_classification_client(settings.CLASSIFICATION_GRPC_ENDPOINT,
                                                         transport=settings.ARENA_CROP_TRANSPORT)
        if not state["client"].connected:
            await state["client"].connect(ready_timeout=30.0)
        if settings.ARENA_CROP_TRANSPORT == "device" and state.get("ring") is None and settings.ARENA_DEVICE != "cpu":
            from .device_transport import DeviceImageRing

            state["ring"] = DeviceImageRing(int(settings.ARENA_DEVICE_RING_SLOTS), 640 * 640 * 3,
                                            device=int(settings.ARENA_GPU))
        log.info("service ready")
        yield
        await state["client"].close()
        state["detector"].close()
        state["decode"].close()

    app = FastAPI(title="Detection Service (MI355X)", version="2.0.0", lifespan=lifespan)
    app.state.arena = state

    async def predict_bytes(data: bytes) -> PredictResponse:
        """The /predict handler on the upload's bytes (shared by FastAPI and the native front end)."""
        rid = new_request_id()
        tm = Timer()
        det_be: DetectorBackend | None = state.get("detector")
        cl: ClassificationClient | None = state.get("client")
        metrics: ArenaMetrics = state["metrics"]
        if det_be is None or cl is None or not cl.connected:
            metrics.observe("unavailable")
            raise HTTPException(status_code=503, detail="Service not ready")
        try:
            state["faults"].check()
            ring = state.get("ring")
            image = None
            if ring is not None:
                h, w = probe_size(data)  # header only: decides the transport before any decode
            else:
                image = await state["decode"].decode(data)
                h, w = image.shape[:2]
            on_device = ring is not None and h * w * 3 <= ring.slot_bytes
            # device transport with a GPU detector: the detector copies the frame it staged for YOLO into a ring
            # slot, device to device inside its batch — the frame crosses PCIe once; with the split decoder
            # (ARENA_NATIVE_DECODE, default on) not even as pixels: the Huffman stage runs on C++ threads and the
            # GPU reconstructs the frame (PIL only for formats the split decoder does not cover)
            slot = ring.try_acquire() if on_device and getattr(det_be, "exports_frames", False) else None
            split = slot is not None and hasattr(det_be, "detect_bytes") and os.environ.get(
                "ARENA_NATIVE_DECODE", "1") != "0"
            if image is None and not split:
                image = await state["decode"].decode(data)
            t_det = Timer()
            if split:
                det_coro = det_be.detect_bytes(data, state["decode"].decode, export_to=ring.slot_ptr(slot))
            elif slot is not None:
                det_coro = det_be.detect(image, export_to=ring.slot_ptr(slot))
            else:
                det_coro = det_be.detect(image)
            det, dtiming = await _detect_holding_slot(det_coro, ring, slot)
            detection_ms = t_det.ms()
            t_cls = Timer()
            boxes = [{"x1": float(d[0]), "y1": float(d[1]), "x2": float(d[2]), "y2": float(d[3]),
                      "confidence": float(d[4]), "class_id": int(d[5])} for d in det]
            crops = [] if on_device else [extract_crop(image, d) for d in det]
            if not boxes:
                if slot is not None:
                    ring.release(slot)
                responses = []
            elif on_device:
                if slot is not None:
                    ref = ring.ref(slot, h, w)
                else:  # no exporting detector (or no free slot before detection): upload the frame once more
                    loop = asyncio.get_running_loop()
                    put = loop.run_in_executor(None, ring.put, image)
                    try:
                        slot, ref = await asyncio.shield(put)
                    except asyncio.CancelledError:
                        # the copy runs on; its slot is released once it lands instead of leaking
                        put.add_done_callback(lambda f: None if f.cancelled() or f.exception() is not None
                                              else ring.release(f.result()[0]))
                        raise
                try:
                    responses = await cl.classify_device(rid, ref, boxes)
                finally:
                    # the answer ends the classification side's use of the frame; after a deadline / cancellation
                    # the classification side drops the abandoned crops before they reach the device
                    # (DeviceClassifier._run), and a batch already on the device that reads a reused slot only
                    # produces answers nobody waits for any more
                    ring.release(slot)
            elif settings.ARENA_FANOUT == "batch":
                responses = await cl.classify_batch(rid, crops, boxes)
            else:
                responses = await cl.classify_parallel(rid, crops, boxes)
            results = []
            for box, r in zip(boxes, responses):
                if r.error:
                    log.warning(f"Classification error for {r.request_id}: {r.error}")
                    continue
                results.append(DetectionWithClassification(
                    detection=DetectionBox(**box),
                    classification=Classification(class_id=r.result.class_id, class_name=r.result.class_name,
                                                  confidence=r.result.confidence)))
            classification_ms = t_cls.ms()
        except Overloaded as e:
            metrics.observe("overloaded")
            raise HTTPException(status_code=503, detail=str(e)) from e
        except HTTPException:
            raise
        except Exception as e:
            metrics.observe("error")
            log.error(f"Predict failed: {e}", extra={"endpoint": "/predict", "status_code": 500})
            raise HTTPException(status_code=500, detail=str(e)) from e
        timing = {"detection_ms": detection_ms, "classification_ms": classification_ms, "total_ms": tm.ms()}
        timing.update({k: float(v) for k, v in dtiming.items()})
        metrics.observe("ok", {k: v for k, v in timing.items() if k.endswith("_ms")}, len(results),
                        int(dtiming.get("batch_size", 1)))
        log.info("Predict complete", extra={"endpoint": "/predict", "latency_ms": timing["total_ms"],
                                            "detections": len(results), "status_code": 200})
        return PredictResponse(request_id=rid, detections=results, timing=timing)

    def healthy() -> bool:
        cl, det = state.get("client"), state.get("detector")
        return device_fault(state) is None and det is not None and cl is not None and cl.connected

    state["predict_bytes"] = predict_bytes
    state["healthy"] = healthy

    @app.post("/predict", response_model=PredictResponse)
    async def predict(request: Request):
        return await predict_bytes(await read_upload(request))

    @app.get("/health", response_model=HealthResponse)
    async def health():
        request_id_var.set(None)
        cl = state.get("client")
        det = state.get("detector")
        if device_fault(state):
            return JSONResponse(status_code=503, content={"status": "unhealthy", "models_loaded": False})
        return HealthResponse(status="healthy", models_loaded=det is not None and cl is not None and cl.connected)

    @app.get("/metrics")
    async def metrics_ep():
        return Response(state["metrics"].render(), media_type="text/plain; version=0.0.4")

    return app


def main() -> None:
    import os

    import uvicorn

    s = Settings.from_env()
    if "PORT" not in os.environ:
        s.PORT = 8200
    uvicorn.run(create_app(s), host=s.HOST, port=s.PORT, log_level="warning", access_log=False)


if __name__ == "__main__":
    main()
