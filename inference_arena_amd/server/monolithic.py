"""Arch A — monolithic service (reference: architectures/monolithic/app/main.py).

One FastAPI process serves ``POST /predict`` (multipart field ``file``) and
``GET /health`` on :8100 with the reference's response schema.  Detection and
classification run in-process — here as one GPU-resident program behind the
native dynamic batcher, so concurrent requests are batched instead of being
serialised by a blocking handler.  ``GET /metrics`` exports Prometheus
metrics.  ``ARENA_DEVICE=cpu`` serves the fp32 CPU reference path instead.

Run: ``python -m inference_arena_amd.server.monolithic`` (PORT, ARENA_GPU, ...).
"""
from __future__ import annotations

import logging
from contextlib import asynccontextmanager

from fastapi import FastAPI, HTTPException, Request
from fastapi.responses import JSONResponse, Response

from ..labels import load_labels
from ..metrics import ArenaMetrics
from ..utils.logging import request_id_var, setup_logging
from ..utils.settings import Settings
from .app_common import DecodePool, FaultInjector, Timer, device_fault, new_request_id, read_upload, to_response
from .backends import Backend, Overloaded, build_backend
from .batching import TooLarge
from .schemas import HealthResponse, PredictResponse

log = logging.getLogger("arena.monolithic")


def create_app(settings: Settings | None = None, backend: Backend | None = None) -> FastAPI:
    settings = settings or Settings.from_env(PORT=None)
    state: dict = {"backend": backend}

    @asynccontextmanager
    async def lifespan(app: FastAPI):
        setup_logging(settings.LOG_LEVEL)
        log.info("starting monolithic service", extra={"port": settings.PORT})
        state["labels"] = load_labels(settings.LABELS_FILE or None)
        state["decode"] = DecodePool(settings.ARENA_DECODE_THREADS)
        state["metrics"] = ArenaMetrics("monolithic", str(settings.ARENA_GPU))
        state["faults"] = FaultInjector(settings.ARENA_FAULT_EVERY)
        if state["backend"] is None:
            state["backend"] = build_backend(settings, arch="monolithic")
        log.info("service ready")
        yield
        log.info("shutting down monolithic service")
        state["backend"].close()
        state["decode"].close()

    app = FastAPI(title="Monolithic Inference Service (MI355X)", version="2.0.0", lifespan=lifespan)
    app.state.arena = state

    @app.post("/predict", response_model=PredictResponse)
    async def predict(request: Request):
        rid = new_request_id()
        tm = Timer()
        be: Backend | None = state.get("backend")
        metrics: ArenaMetrics = state["metrics"]
        if be is None or not be.ready():
            metrics.observe("unavailable")
            raise HTTPException(status_code=503, detail="Service not ready")
        data = await read_upload(request)
        try:
            state["faults"].check()
            t_dec = Timer()
            image = await state["decode"].decode(data)
            decode_ms = t_dec.ms()
            res, timing = await be.infer(image)
        except Overloaded as e:
            metrics.observe("overloaded")
            raise HTTPException(status_code=503, detail=str(e)) from e
        except TooLarge as e:
            metrics.observe("too_large")
            raise HTTPException(status_code=413, detail=str(e)) from e
        except Exception as e:  # reference: any failure -> 500 with detail=str(e)
            metrics.observe("error")
            log.error(f"Predict failed: {e}", extra={"endpoint": "/predict", "status_code": 500})
            raise HTTPException(status_code=500, detail=str(e)) from e
        timing = dict(timing)
        timing["decode_ms"] = decode_ms
        timing["total_ms"] = tm.ms()
        metrics.observe("ok", {k: v for k, v in timing.items() if k.endswith("_ms")}, len(res),
                        int(timing.get("batch_size", 1)))
        log.info("Predict complete", extra={"endpoint": "/predict", "latency_ms": timing["total_ms"],
                                            "detections": len(res), "status_code": 200})
        return to_response(rid, res, state["labels"], timing, settings.ARENA_CONFIDENCE or "logit")

    @app.get("/health", response_model=HealthResponse)
    async def health():
        request_id_var.set(None)
        be = state.get("backend")
        if device_fault(state):
            # device fault: 503 so probes / the replica router take this instance out of rotation
            return JSONResponse(status_code=503, content={"status": "unhealthy", "models_loaded": False})
        return HealthResponse(status="healthy", models_loaded=be is not None and be.ready())

    @app.get("/metrics")
    async def metrics():
        be = state.get("backend")
        m: ArenaMetrics = state["metrics"]
        if be is not None:
            st = be.stats()
            if "queue_depth" in st:
                m.queue.labels(m.arch, m.gpu).set(st["queue_depth"])
        return Response(m.render(), media_type="text/plain; version=0.0.4")

    return app


def main() -> None:
    import uvicorn

    s = Settings.from_env()
    if "PORT" not in __import__("os").environ:
        s.PORT = 8100
    uvicorn.run(create_app(s), host=s.HOST, port=s.PORT, log_level="warning", access_log=False)


if __name__ == "__main__":
    main()
