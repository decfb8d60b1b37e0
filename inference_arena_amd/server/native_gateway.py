"""Arch C — native gateway (``ARENA_GATEWAY_NATIVE=1``): the gateway's ``POST /predict`` served by the C++ front
end in proxy mode (csrc/runtime/http_front.h ``upstream_*``, csrc/runtime/kserve.h ``KServeProxy``).

Reference: architectures/triton/gateway/app/main.py:98-155 / pipeline.py:102-207 (a FastAPI gateway calling
Triton's ModelInfer over gRPC).  Round 4 measured the Python gateway + the model server's Python gRPC servicer as
7 of the 12 ms mean RPC at 100 users and 9.5 CPUs of model-server Python.  Here no Python
runs per request on either side: the gateway's epoll threads parse the upload, a pool of keep-alive connections
forwards it as a KServe-v2 REST infer request (binary tensor extension) to the model server's native endpoint
(``ARENA_KSERVE_NATIVE_PORT``, server/model_server.py), whose C++ front end decodes, batches and runs the
``arena_pipeline`` ensemble and answers binary output tensors; the gateway turns them into the reference JSON.
The gRPC KServe endpoint (:8001) and the Python REST app (:8000) stay for compatibility.

Run: ``python -m inference_arena_amd.server.native_gateway`` (PORT, TRITON_HTTP_ENDPOINT host:port,
ARENA_GATEWAY_CONNS, ARENA_HTTP_THREADS, ARENA_CONFIDENCE).
"""
from __future__ import annotations

import logging
import os
import signal
import threading
import time
import urllib.request

from prometheus_client import CollectorRegistry, generate_latest

from ..labels import load_labels
from ..utils.logging import setup_logging
from ..utils.settings import Settings
from .native_front import _Collector, _http_timeouts

log = logging.getLogger("arena.native_gateway")


class NativeGateway:
    """The gateway's native HTTP server, forwarding to a model server's native KServe endpoint."""

    def __init__(self, labels: list[str], *, upstream: str, port: int = 8300, host: str = "0.0.0.0",
                 model: str = "arena_pipeline", conns: int = 256, io_threads: int = 4, softmax: bool = False,
                 replica_tag: str = ""):
        from ..ops import native

        # "host:port" or "host:port,host:port,...": one model server per GPU, least-outstanding first
        self.upstreams = []
        for item in (u.strip() for u in upstream.split(",")):
            if item:
                uh, _, up = item.rpartition(":")
                self.upstreams.append((uh or "127.0.0.1", int(up)))
        if not self.upstreams:
            raise ValueError("native gateway: no upstream")
        self.upstream = self.upstreams[0]
        self.model = model
        self.batcher = None
        self.fe = native().http_proxy_front(list(labels), {
            "host": host, "port": int(port), "io_threads": int(io_threads), "softmax_confidence": bool(softmax),
            "replica_tag": str(replica_tag), "upstream_host": self.upstream[0], "upstream_port": self.upstream[1],
            "upstreams": ",".join(f"{h}:{p}" for h, p in self.upstreams[1:]),
            "upstream_model": model, "upstream_conns": int(conns), **_http_timeouts()})
        self.fe.set_healthy(False)
        self.extra_metrics = ""
        self.registry = CollectorRegistry()
        self.registry.register(_Collector(self, "triton", "-"))
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._refresh, name="native-gateway-metrics", daemon=True)
        self._thread.start()

    @property
    def port(self) -> int:
        return self.fe.port

    def stats(self) -> dict:
        return self.fe.stats()

    def upstream_forwarded(self) -> list[int]:
        """Requests forwarded to each upstream so far (the proxy's least-outstanding spread)."""
        return list(self.fe.upstream_forwarded())

    def upstream_ready(self) -> bool:
        for h, p in self.upstreams:
            try:
                with urllib.request.urlopen(f"http://{h}:{p}/v2/models/{self.model}/ready", timeout=2) as r:
                    if r.status != 200:
                        return False
            except OSError:
                return False
        return True

    def wait_ready(self, timeout_s: float = 60.0) -> bool:
        """Backoff capped at 10 s (reference triton_client.py wait_for_server_ready); turns healthy once the
        model server's ensemble answers ready."""
        t0, delay = time.monotonic(), 0.25
        while time.monotonic() - t0 < timeout_s:
            if self.upstream_ready():
                self.fe.set_healthy(True)
                return True
            time.sleep(delay)
            delay = min(delay * 2, 10.0)
        return False

    def _refresh(self) -> None:
        while not self._stop.is_set():
            try:
                self.fe.set_metrics_text(generate_latest(self.registry).decode() + self.extra_metrics)
            except Exception as e:  # noqa: BLE001
                log.warning(f"metrics refresh failed: {e}")
            self._stop.wait(1.0)

    def close(self) -> None:
        self._stop.set()
        self.fe.stop()


def serve(settings: Settings | None = None, replica_tag: str = "") -> int:
    settings = settings or Settings.from_env()
    setup_logging(settings.LOG_LEVEL)
    upstream = os.environ.get("TRITON_HTTP_ENDPOINT", "127.0.0.1:8004")
    port = int(os.environ.get("PORT", "8300"))
    # ARENA_LOCAL_WORLD gateway processes (one per GPU, SO_REUSEPORT on :8300) each pin to their GPU's CPU share
    world = int(os.environ.get("ARENA_LOCAL_WORLD", "1") or 1)
    io_threads = int(os.environ.get("ARENA_HTTP_THREADS", "4"))
    host = None
    if world > 1:
        from ..parallel.affinity import rank_host_setup

        host = rank_host_setup(int(os.environ.get("ARENA_REPLICA_GPU", replica_tag or "0") or 0), world)
        io_threads = host["plan"]["http_io"]
    gw = NativeGateway(load_labels(settings.LABELS_FILE or None), upstream=upstream, port=port,
                       # one upstream request in flight per connection: 64 capped the arm at 64 requests in the
                       # model server, so 100 users measured like 75 (protocol_r6: 7038 -> 7100 req/s)
                       conns=int(os.environ.get("ARENA_GATEWAY_CONNS", "256")), io_threads=io_threads,
                       softmax=(settings.ARENA_CONFIDENCE or "logit") == "softmax", replica_tag=replica_tag)
    if host is not None:
        from ..parallel.affinity import rank_info_metrics

        gw.extra_metrics = rank_info_metrics(dict(host, plan={"http_io": io_threads}), "gateway")
        log.info(f"gateway rank {replica_tag}: cpus {host['cpus']}, usable {host['usable_cpus']}, io {io_threads}")
    if not gw.wait_ready(float(settings.TRITON_TIMEOUT_SECONDS)):
        log.error(f"model server native endpoint {upstream} not ready")
        gw.close()
        return 1
    log.info("native gateway ready", extra={"port": gw.port, "upstream": upstream})
    done = threading.Event()
    if threading.current_thread() is threading.main_thread():
        for sig in (signal.SIGTERM, signal.SIGINT):
            signal.signal(sig, lambda *_: done.set())
    while not done.wait(0.5):
        pass
    gw.close()
    return 0


if __name__ == "__main__":
    raise SystemExit(serve())
