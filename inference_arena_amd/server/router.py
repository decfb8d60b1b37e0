"""Least-outstanding-requests HTTP router over per-GPU replicas.

For deployments where replicas cannot share a port (``--port-stride``, or
replicas on several hosts), this front forwards each request to the replica
with the fewest requests in flight (ties -> round robin), which keeps every
GPU's dynamic batcher fed evenly under skewed load.  A replica that refuses
connections is skipped until its next health probe succeeds.

Run: ``python -m inference_arena_amd.server.router --port 8100 --backends 127.0.0.1:8110,127.0.0.1:8111``.
"""
from __future__ import annotations

import argparse
import asyncio
import itertools

from fastapi import Request


class Router:
    def __init__(self, backends: list[str], timeout_s: float = 60.0, probe_s: float = 2.0):
        self.backends = [b if b.startswith("http") else f"http://{b}" for b in backends]
        self.inflight = {b: 0 for b in self.backends}
        self.healthy = {b: True for b in self.backends}
        self.served = {b: 0 for b in self.backends}
        self._rr = itertools.count()
        self.timeout_s = timeout_s
        self.probe_s = probe_s
        self.session = None
        self._probe_task = None

    def pick(self) -> str:
        cands = [b for b in self.backends if self.healthy[b]] or list(self.backends)
        low = min(self.inflight[b] for b in cands)
        best = [b for b in cands if self.inflight[b] == low]
        return best[next(self._rr) % len(best)]

    async def start(self):
        import aiohttp

        self.session = aiohttp.ClientSession(connector=aiohttp.TCPConnector(limit=0),
                                             timeout=aiohttp.ClientTimeout(total=self.timeout_s))
        self._probe_task = asyncio.create_task(self._probe())

    async def close(self):
        if self._probe_task:
            self._probe_task.cancel()
        if self.session:
            await self.session.close()

    async def _probe(self):
        import aiohttp

        while True:
            for b in self.backends:
                try:
                    async with self.session.get(f"{b}/health") as r:
                        self.healthy[b] = r.status == 200
                except (aiohttp.ClientError, asyncio.TimeoutError):
                    self.healthy[b] = False
            await asyncio.sleep(self.probe_s)

    async def forward(self, method: str, path: str, body: bytes, headers: dict) -> tuple[int, bytes, dict]:
        import aiohttp

        tried = set()
        while True:
            b = self.pick()
            tried.add(b)
            self.inflight[b] += 1
            try:
                async with self.session.request(method, f"{b}{path}", data=body, headers=headers) as r:
                    data = await r.read()
                    self.served[b] += 1
                    keep = {k: v for k, v in r.headers.items()
                            if k.lower() in ("content-type", "x-arena-replica")}
                    return r.status, data, keep
            except aiohttp.ClientConnectionError:
                self.healthy[b] = False
                if len(tried) >= len(self.backends):
                    return 502, b'{"detail":"no replica reachable"}', {"content-type": "application/json"}
            finally:
                self.inflight[b] -= 1


def create_app(backends: list[str]):
    from contextlib import asynccontextmanager

    from fastapi import FastAPI
    from fastapi.responses import JSONResponse, Response

    router = Router(backends)

    @asynccontextmanager
    async def lifespan(app):
        await router.start()
        yield
        await router.close()

    app = FastAPI(title="arena replica router", lifespan=lifespan)
    app.state.router = router

    @app.get("/router/stats")
    async def stats():
        return {"inflight": router.inflight, "healthy": router.healthy, "served": router.served}

    @app.get("/health")
    async def health():
        ok = any(router.healthy.values())
        return JSONResponse({"status": "healthy" if ok else "unhealthy", "models_loaded": ok},
                            status_code=200 if ok else 503)

    @app.api_route("/{path:path}", methods=["GET", "POST"])
    async def proxy(path: str, request: Request):
        hdr = {k: v for k, v in request.headers.items() if k.lower() in ("content-type",)}
        st, data, h = await router.forward(request.method, "/" + path, await request.body(), hdr)
        return Response(data, status_code=st, headers=h)

    return app


def main(argv=None) -> int:
    import uvicorn

    ap = argparse.ArgumentParser()
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=8100)
    ap.add_argument("--backends", required=True, help="comma-separated host:port list")
    a = ap.parse_args(argv)
    uvicorn.run(create_app(a.backends.split(",")), host=a.host, port=a.port, log_level="warning", access_log=False)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
