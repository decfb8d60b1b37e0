"""Native HTTP front end in handler mode for the Python-orchestrated arms.

The microservices detection service (server/detection_service.py) and the model-server gateway
(server/gateway.py) orchestrate each request in Python (decode, detector batcher, gRPC fan-out to the
classification service / KServe calls), but the HTTP layer under them does not need to be Python.
uvicorn/h11 + starlette + multipart parsing cost ~0.7-1.4 ms of interpreter time per request
(tools/http_overhead.py), which capped one process of those arms at ~700-900 req/s
(profiles/serving_r2b).  Here the C++ epoll front end (csrc/runtime/http_front.cpp, handler mode)
parses HTTP/1.1 and multipart and queues the upload bytes; one Python thread drains the queue
(``take``, GIL released while waiting) into the arm's asyncio loop, where the same
``predict_bytes`` coroutine the FastAPI route uses runs; the JSON goes back with ``complete``.

Same contract as the FastAPI apps (reference architectures/microservices/detection/app/main.py,
architectures/triton/gateway/app/main.py): ``POST /predict`` -> PredictResponse JSON, errors as
``{"detail": ...}`` with the handler's status code, ``GET /health`` (503 once unhealthy),
``GET /metrics`` (the arm's ArenaMetrics text, refreshed every second).

Used by ``server/replica.py`` when ``ARENA_NATIVE_HTTP=1`` for ``--arch detection|gateway``.
"""
from __future__ import annotations

import asyncio
import json
import logging
import signal
import threading

from fastapi import HTTPException

log = logging.getLogger("arena.native_handler")


class NativeHandlerServer:
    """The native front end (handler mode) driving ``predict_bytes`` on an asyncio loop."""

    def __init__(self, predict_bytes, *, port: int, host: str = "0.0.0.0", io_threads: int = 2,
                 replica_tag: str = "", max_queue: int = 4096, reuse_port: bool = True):
        from ..ops import native

        self.predict_bytes = predict_bytes
        self.fe = native().HttpFrontEnd({"host": host, "port": int(port), "io_threads": int(io_threads),
                                         "replica_tag": str(replica_tag), "max_queue": int(max_queue),
                                         "reuse_port": bool(reuse_port)})
        self._stop = threading.Event()
        self._taker: threading.Thread | None = None
        self.inflight = 0

    @property
    def port(self) -> int:
        return self.fe.port

    def set_healthy(self, ok: bool) -> None:
        self.fe.set_healthy(bool(ok))

    def set_metrics_text(self, text: str) -> None:
        self.fe.set_metrics_text(text)

    def stats(self) -> dict:
        return self.fe.stats()

    async def _one(self, key: int, data: bytes) -> None:
        self.inflight += 1
        try:
            resp = await self.predict_bytes(data)
            body, code, n = resp.model_dump_json(), 200, len(resp.detections)
        except HTTPException as e:
            body, code, n = json.dumps({"detail": e.detail}), int(e.status_code), 0
        except Exception as e:  # noqa: BLE001 - every request gets an answer
            body, code, n = json.dumps({"detail": str(e)}), 500, 0
        finally:
            self.inflight -= 1
        self.fe.complete(key, code, body, n)

    def start(self, loop: asyncio.AbstractEventLoop) -> None:
        """Start the thread that moves queued uploads onto ``loop``."""

        def spawn(items):
            for key, data in items:
                loop.create_task(self._one(key, data))

        def taker():
            while not self._stop.is_set():
                items = self.fe.take(256, 100)
                if items:
                    try:
                        loop.call_soon_threadsafe(spawn, items)
                    except RuntimeError:  # loop closed during shutdown
                        return

        self._taker = threading.Thread(target=taker, name="native-handler-take", daemon=True)
        self._taker.start()

    def drain(self) -> None:
        """Stop accepting connections; open connections and queued requests are still answered."""
        self.fe.drain()

    def pending(self) -> int:
        return int(self.fe.handler_pending())

    def close(self) -> None:
        self._stop.set()
        self.fe.stop()
        if self._taker is not None:
            self._taker.join(2.0)


async def serve_app(app, *, port: int, host: str = "0.0.0.0", replica_tag: str = "", io_threads: int = 2,
                    stop: asyncio.Event | None = None, on_ready=None, reuse_port: bool = True,
                    drain_s: float = 10.0) -> int:
    """Run a FastAPI arm app (its lifespan, then ``state['predict_bytes']``) behind the native front end until
    ``stop`` is set or SIGTERM/SIGINT; returns 3 after a device fault (the replica supervisor restarts it)."""
    from .app_common import device_fault

    state = app.state.arena
    stop = stop or asyncio.Event()
    loop = asyncio.get_running_loop()
    if threading.current_thread() is threading.main_thread():
        for sig in (signal.SIGTERM, signal.SIGINT):
            loop.add_signal_handler(sig, stop.set)
    rc = 0
    async with app.router.lifespan_context(app):
        srv = NativeHandlerServer(state["predict_bytes"], port=port, host=host, io_threads=io_threads,
                                  replica_tag=replica_tag, reuse_port=reuse_port)
        srv.start(loop)
        log.info("native handler front end ready", extra={"port": srv.port})
        if on_ready is not None:
            on_ready(srv)
        healthy = state.get("healthy", lambda: True)
        metrics = state.get("metrics")
        ticks = 0
        try:
            while not stop.is_set():
                try:
                    await asyncio.wait_for(stop.wait(), 0.2)
                except asyncio.TimeoutError:
                    pass
                srv.set_healthy(bool(healthy()))
                if device_fault(state):
                    log.error("device fault; leaving rotation and exiting for a restart")
                    srv.set_healthy(False)
                    rc = 3
                    break
                ticks += 1
                if metrics is not None and ticks % 5 == 1:
                    srv.set_metrics_text(metrics.render().decode())
        finally:
            # like uvicorn's shutdown: leave the port first (an SO_REUSEPORT peer takes new connections), answer
            # what is queued or in the handler (bounded), then stop the I/O threads
            srv.drain()
            for _ in range(int(drain_s / 0.02)):
                if srv.pending() == 0:
                    break
                await asyncio.sleep(0.02)
            srv.close()
    return rc
