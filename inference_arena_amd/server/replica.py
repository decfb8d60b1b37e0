"""One serving replica per GPU (data parallelism for the serving topologies).

Launched by ``parallel.replicas.launch`` with torchrun-style env (RANK,
WORLD_SIZE, LOCAL_RANK, MASTER_ADDR/PORT).  Start-up:

1. join the process group (``nccl`` = RCCL over xGMI on MI355X; ``gloo``
   for the CPU device),
2. rank 0 produces the folded weight blob of the arm's program and
   broadcasts it in one collective; every replica serves identical weights,
3. bind the HTTP port with ``SO_REUSEPORT`` — all replicas share one port
   and the kernel spreads connections over them (no proxy hop), or
   ``--port-stride`` gives each replica its own port behind ``router.py``,
4. serve the arm (monolithic / detection / gateway) on GPU ``LOCAL_RANK``.

Each response carries ``x-arena-replica: <rank>``.

Failover (SURVEY.md §5 failure detection): a watchdog polls the arm's device
fault state; on a HIP fault the replica stops accepting (closes its listening
socket, drains in-flight requests) and exits with code 3, and the supervisor
in ``parallel.replicas`` starts a fresh child process for the same GPU (never
an exec of the faulted process).  A restarted replica runs with world size 1
(``ARENA_REPLICA_GPU`` names its device) and derives the same seeded weights.
"""
from __future__ import annotations

import argparse
import asyncio
import os
import socket


def _socket(host: str, port: int, reuse_port: bool) -> socket.socket:
    s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    if reuse_port:
        s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEPORT, 1)
    # accepted connections inherit TCP_NODELAY on Linux; without it a response written
    # as header + body segments waits on the client's delayed ACK (~40 ms per request)
    s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
    s.bind((host, port))
    s.listen(2048)
    s.setblocking(False)
    return s


class ReplicaTag:
    """Pure-ASGI wrapper adding ``x-arena-replica`` to every HTTP response (a
    Starlette BaseHTTPMiddleware costs ~1 ms per request)."""

    def __init__(self, app, rank: int):
        self.app = app
        self.tag = str(rank).encode()

    async def __call__(self, scope, receive, send):
        if scope["type"] != "http":
            return await self.app(scope, receive, send)

        async def send_tagged(msg):
            if msg["type"] == "http.response.start":
                msg = dict(msg)
                msg["headers"] = list(msg.get("headers", [])) + [(b"x-arena-replica", self.tag)]
            await send(msg)

        await self.app(scope, receive, send_tagged)


def build_app(arch: str, settings, info):
    """The arm's FastAPI app with weights broadcast from rank 0."""
    import numpy as np

    from ..models.zoo import resolve_models
    from ..parallel import dist as D

    if arch == "monolithic":
        from .monolithic import create_app

        if settings.ARENA_DEVICE == "cpu":
            from .backends import build_backend

            backend = build_backend(settings)
            D.broadcast_object(None, info)
        else:
            from ..config import get_triton_config
            from ..engine.plans import plan_pipeline
            from .backends import GpuBatchedBackend

            yolo, mnet = resolve_models(settings.MODELS_DIR, int(settings.ARENA_WEIGHT_SEED))
            from ..engine.pipeline import resolve_dtype

            blob = plan_pipeline(yolo, mnet, conf_thr=0.0, iou_thr=0.0,  # weights only: thresholds unused
                                 dtype=resolve_dtype()).weights if info.is_main else None
            blob = D.broadcast_blob(blob, info)
            db = get_triton_config().get("dynamic_batching", {}) or {}
            backend = GpuBatchedBackend(yolo, mnet, device=int(settings.ARENA_GPU),  # one GPU per replica
                                        instances=int(settings.ARENA_INSTANCES),
                                        max_batch=int(settings.ARENA_MAX_BATCH),
                                        preferred=list(db.get("preferred_batch_size", [])),
                                        max_queue_delay_us=int(settings.ARENA_QUEUE_DELAY_US),
                                        weights=np.ascontiguousarray(blob))
        return create_app(settings, backend)
    if arch == "detection":
        from .detection_service import create_app

        return create_app(settings)
    if arch == "gateway":
        from .gateway import create_app

        return create_app(settings)
    raise ValueError(f"unknown arch '{arch}'")


def _serve_native(settings, info, port: int, rank: int | None = None) -> int:
    """``ARENA_NATIVE_HTTP=1``: the monolithic replica behind the native C++ front end
    (server/native_front.py) with rank 0's broadcast weights; exits 3 after a device fault."""
    import numpy as np

    from ..engine.pipeline import resolve_dtype
    from ..engine.plans import plan_pipeline
    from ..models.zoo import resolve_models
    from ..parallel import dist as D
    from .native_front import serve

    if settings.ARENA_DEVICE == "fake":  # host-only stand-in engine: no weights to broadcast
        blob = None
    else:
        yolo, mnet = resolve_models(settings.MODELS_DIR, int(settings.ARENA_WEIGHT_SEED))
        blob = plan_pipeline(yolo, mnet, conf_thr=0.0, iou_thr=0.0,  # weights only: thresholds unused
                             dtype=resolve_dtype()).weights if info.is_main else None
        blob = np.ascontiguousarray(D.broadcast_blob(blob, info))
    D.barrier(info)
    D.shutdown(info)
    settings.PORT = port
    return serve(settings, weights=blob, replica_tag=str(info.rank if rank is None else rank),
                 devices=[int(settings.ARENA_GPU)])


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="monolithic", choices=["monolithic", "detection", "gateway"])
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=8100)
    ap.add_argument("--port-stride", type=int, default=0, help="0: shared SO_REUSEPORT port; k: port + k*rank")
    a = ap.parse_args(argv)

    import uvicorn

    from ..parallel import dist as D
    from ..utils.settings import Settings

    import os

    from .decode_pool import prestart

    prestart()  # decode-worker fork server before any GPU initialisation (server/decode_pool.py)
    settings = Settings.from_env()
    per_gpu = max(1, int(os.environ.get("ARENA_PROCS_PER_GPU", "1")))
    backend = "gloo" if settings.ARENA_DEVICE in ("cpu", "fake") or per_gpu > 1 else None
    info = D.init_from_env(backend)
    if settings.ARENA_DEVICE != "cpu":
        override = os.environ.get("ARENA_REPLICA_GPU")
        first = int(os.environ.get("ARENA_FIRST_GPU", "0"))
        settings.ARENA_GPU = int(override) if override else first + info.local_rank // per_gpu
        if backend == "gloo" and settings.ARENA_DEVICE == "gpu":
            import torch

            torch.cuda.set_device(settings.ARENA_GPU)
    # a restarted replica runs in a one-process world (RANK 0) but keeps its original port and tag
    rank = int(os.environ.get("ARENA_REPLICA_RANK", info.rank))
    if a.arch == "monolithic" and settings.ARENA_DEVICE != "cpu" and os.environ.get("ARENA_NATIVE_HTTP") == "1":
        return _serve_native(settings, info, a.port + a.port_stride * rank, rank)
    if a.arch == "gateway" and os.environ.get("ARENA_GATEWAY_NATIVE") == "1":
        # the gateway's request path entirely in C++: proxy to the model server's native KServe endpoint
        # (server/native_gateway.py; TRITON_HTTP_ENDPOINT)
        from .native_gateway import serve as serve_gateway

        D.barrier(info)
        D.shutdown(info)
        os.environ["PORT"] = str(a.port + a.port_stride * rank)
        return serve_gateway(settings, replica_tag=str(rank))
    app = build_app(a.arch, settings, info)
    D.barrier(info)
    D.shutdown(info)  # the group is only needed for start-up

    port = a.port + a.port_stride * rank
    if a.arch in ("detection", "gateway") and os.environ.get("ARENA_NATIVE_HTTP") == "1":
        # native HTTP/multipart layer, the arm's request handler stays in Python (server/native_handler.py)
        from .native_handler import serve_app

        rc = asyncio.run(serve_app(app, port=port, host=a.host, replica_tag=str(rank),
                                   io_threads=int(os.environ.get("ARENA_HTTP_THREADS", "2")),
                                   reuse_port=a.port_stride == 0))
        if rc and os.environ.get("ARENA_EXIT_ON_FAULT", "1") == "1":
            print(f"replica {info.rank}: device fault, exiting for restart", flush=True)
            return 3
        return 0
    sock = _socket(a.host, port, reuse_port=a.port_stride == 0)
    server = uvicorn.Server(uvicorn.Config(ReplicaTag(app, rank), log_level="warning", access_log=False))
    fault: list[str] = []

    async def watchdog():
        from .app_common import device_fault

        while not server.should_exit:
            await asyncio.sleep(0.2)
            err = device_fault(getattr(app.state, "arena", {}) or {})
            if err:
                fault.append(err)
                # uvicorn's shutdown first closes the listening socket (the kernel stops routing new
                # connections to this process), then drains in-flight requests and returns
                server.should_exit = True
                return

    async def serve():
        task = asyncio.create_task(watchdog())
        await server.serve(sockets=[sock])
        task.cancel()

    asyncio.run(serve())
    if fault and os.environ.get("ARENA_EXIT_ON_FAULT", "1") == "1":
        print(f"replica {info.rank}: device fault, exiting for restart: {fault[0]}", flush=True)
        return 3
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
