#!/usr/bin/env python3
"""Per-request host cost of the HTTP front end (no GPU): the monolithic app with a stub backend.

Starts ``server.monolithic.create_app`` under uvicorn in a child process with a backend that answers
instantly with a fixed 4-detection result, drives it with closed-loop aiohttp clients in separate
processes, and reports req/s and latency — the ceiling the Python front end (multipart parse, decode
hand-off, response building, logging, metrics) puts on a serving process.  ``--profile`` writes the
server's cProfile top functions.

    python tools/http_overhead.py --seconds 8 --users 64 --clients 2 [--decode-procs 4] [--profile out.txt]
"""
from __future__ import annotations

import argparse
import asyncio
import json
import multiprocessing as mp
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


class StubBackend:
    name = "stub"

    def ready(self):
        return True

    async def infer(self, image):
        import numpy as np

        from inference_arena_amd.engine.pipeline import ImageResult

        n = 4
        res = ImageResult(boxes=np.tile(np.array([[10, 20, 110, 220]], np.float32), (n, 1)),
                          scores=np.full(n, 0.9, np.float32), classes=np.zeros(n, np.int32),
                          topk_idx=np.tile(np.arange(5, dtype=np.int32), (n, 1)),
                          topk_logit=np.ones((n, 5), np.float32), topk_prob=np.full((n, 5), 0.2, np.float32),
                          det_count=n)
        return res, {"queue_ms": 0.1, "gpu_ms": 1.0, "batch_size": 1.0, "detection_ms": 1.1,
                     "classification_ms": 0.0, "inference_ms": 1.2}

    def stats(self):
        return {}

    def close(self):
        pass


def _serve_native(port: int, seconds: float, decode_procs: int) -> None:  # pragma: no cover - child process
    """The native front end (csrc/runtime/http_front.h) over the host-only EchoInstance."""
    from inference_arena_amd.labels import load_labels
    from inference_arena_amd.ops import native
    from inference_arena_amd.server.native_front import NativeFrontEnd

    C = native()
    batcher = C.DynamicBatcher([C.EchoInstance(4, 32, 4)], {"max_batch": 32, "max_queue_delay_us": 200})
    fe = NativeFrontEnd(batcher, load_labels(None), port=port, host="127.0.0.1", io_threads=4,
                        decode_procs=max(1, decode_procs))
    time.sleep(seconds)
    fe.close()
    batcher.shutdown()


def _stub_classifier(gport: int, seconds: float) -> None:  # pragma: no cover - child process
    import numpy as np

    from inference_arena_amd.server.classification_service import start_server
    from inference_arena_amd.server.service_backends import ClassifierBackend
    from inference_arena_amd.utils.settings import Settings

    class StubClassifier(ClassifierBackend):
        async def classify(self, crop):
            return (np.arange(5, dtype=np.int32), np.array([5, 4, 3, 2, 1], np.float32),
                    np.array([0.6, 0.2, 0.1, 0.05, 0.05], np.float32))

    async def run():
        srv = await start_server(Settings(LOG_LEVEL="WARNING", HOST="127.0.0.1"), StubClassifier(), port=gport)
        await asyncio.sleep(seconds)
        await srv[0].stop(0)

    asyncio.run(run())


def _serve_detection(port: int, seconds: float, native_front: bool) -> None:  # pragma: no cover - child process
    """The microservices detection service (stub detector: 4 boxes) fanning out to a stub classification gRPC
    service (its own process); FastAPI/uvicorn or the native front end in handler mode (server/native_handler.py)."""
    import socket
    import threading

    import numpy as np

    from inference_arena_amd.server.detection_service import create_app
    from inference_arena_amd.server.service_backends import DetectorBackend
    from inference_arena_amd.utils.settings import Settings

    class StubDetector(DetectorBackend):
        async def detect(self, image):
            return np.tile(np.array([[10, 20, 110, 220, 0.9, 1]], np.float32), (4, 1)), {"batch_size": 1.0}

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        gport = sk.getsockname()[1]
    cls = mp.get_context("spawn").Process(target=_stub_classifier, args=(gport, seconds + 5), daemon=True)
    cls.start()
    s = Settings.from_env(PORT=port)
    s.CLASSIFICATION_GRPC_ENDPOINT = f"127.0.0.1:{gport}"
    s.ARENA_FANOUT, s.ARENA_CROP_TRANSPORT, s.LOG_LEVEL = "batch", "raw", "WARNING"
    app = create_app(s, detector=StubDetector())
    if native_front:
        from inference_arena_amd.server.native_handler import serve_app

        async def run():
            stop = asyncio.Event()
            asyncio.get_running_loop().call_later(seconds, stop.set)
            await serve_app(app, port=port, host="127.0.0.1", stop=stop)

        asyncio.run(run())
    else:
        import uvicorn

        server = uvicorn.Server(uvicorn.Config(app, host="127.0.0.1", port=port, log_level="warning",
                                               access_log=False))
        threading.Timer(seconds, lambda: setattr(server, "should_exit", True)).start()
        server.run()


def _serve(port: int, profile: str | None, seconds: float) -> None:  # pragma: no cover - child process
    import uvicorn

    from inference_arena_amd.server.monolithic import create_app
    from inference_arena_amd.utils.settings import Settings

    app = create_app(Settings.from_env(PORT=port), backend=StubBackend())
    cfg = uvicorn.Config(app, host="127.0.0.1", port=port, log_level="warning", access_log=False)
    server = uvicorn.Server(cfg)
    if profile:
        import cProfile
        import pstats
        import threading

        prof = cProfile.Profile()
        threading.Timer(seconds, lambda: setattr(server, "should_exit", True)).start()
        prof.enable()
        server.run()
        prof.disable()
        with open(profile, "w") as f:
            pstats.Stats(prof, stream=f).sort_stats("tottime").print_stats(40)
    else:
        server.run()


def _client(port: int, users: int, seconds: float, jpeg: bytes, q) -> None:  # pragma: no cover - child
    import aiohttp

    async def run():
        lat = []
        stop = time.perf_counter() + seconds
        url = f"http://127.0.0.1:{port}/predict"
        async with aiohttp.ClientSession(connector=aiohttp.TCPConnector(limit=users)) as s:
            async def user():
                while time.perf_counter() < stop:
                    form = aiohttp.FormData()
                    form.add_field("file", jpeg, filename="x.jpg", content_type="image/jpeg")
                    t = time.perf_counter()
                    async with s.post(url, data=form) as r:
                        await r.read()
                        if r.status == 200:
                            lat.append(time.perf_counter() - t)
            await asyncio.gather(*[user() for _ in range(users)])
        return lat
    q.put(asyncio.run(run()))


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=8)
    ap.add_argument("--users", type=int, default=64, help="concurrent connections per client process")
    ap.add_argument("--clients", type=int, default=2)
    ap.add_argument("--port", type=int, default=8190)
    ap.add_argument("--decode-procs", type=int, default=0)
    ap.add_argument("--profile", default=None)
    ap.add_argument("--tiny", action="store_true", help="a 32x32 upload: decode cost ~0, isolates the HTTP path")
    ap.add_argument("--native", action="store_true", help="the native C++ front end instead of FastAPI")
    ap.add_argument("--arm", default="monolithic", choices=["monolithic", "detection"],
                    help="detection: the microservices detection service + stub gRPC classifier")
    a = ap.parse_args(argv)
    os.environ["ARENA_DECODE_PROCS"] = str(a.decode_procs)
    os.environ.setdefault("LOG_LEVEL", "INFO")
    from inference_arena_amd.data.curator import workload_images
    from inference_arena_amd.data.synthetic import encode_jpeg

    img = workload_images(1)[0]
    jpeg = encode_jpeg(img[:32, :32].copy() if a.tiny else img, 90)
    ctx = mp.get_context("spawn")
    if a.arm == "detection":
        srv = ctx.Process(target=_serve_detection, args=(a.port, a.seconds + 8, a.native))
    elif a.native:
        srv = ctx.Process(target=_serve_native, args=(a.port, a.seconds + 8, a.decode_procs or 4))
    else:  # not daemonic: it spawns decode workers
        srv = ctx.Process(target=_serve, args=(a.port, a.profile, a.seconds + 6))
    srv.start()
    import urllib.request

    for _ in range(120):
        try:
            urllib.request.urlopen(f"http://127.0.0.1:{a.port}/health", timeout=1)
            break
        except OSError:
            time.sleep(0.25)
    q = ctx.Queue()
    warm = ctx.Process(target=_client, args=(a.port, 4, 1.0, jpeg, q))
    warm.start()
    q.get()
    warm.join()
    cl = [ctx.Process(target=_client, args=(a.port, a.users, a.seconds, jpeg, q)) for _ in range(a.clients)]
    for c in cl:
        c.start()
    lat = []
    for _ in cl:
        lat += q.get()
    for c in cl:
        c.join()
    import numpy as np

    out = {"req_s": round(len(lat) / a.seconds, 1), "p50_ms": round(float(np.percentile(lat, 50)) * 1e3, 2),
           "p99_ms": round(float(np.percentile(lat, 99)) * 1e3, 2), "users": a.users * a.clients,
           "decode_procs": a.decode_procs, "front_end": "native" if a.native else "fastapi", "tiny": a.tiny, "arm": a.arm}
    print(json.dumps(out), flush=True)
    if a.profile:
        srv.join(timeout=a.seconds + 30)
    srv.terminate()
    srv.join(timeout=5)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
