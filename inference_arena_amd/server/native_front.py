"""Monolithic arm with the native HTTP front end (csrc/runtime/http_front.h).

Same contract as ``server/monolithic.py`` (reference architectures/monolithic/app/main.py: ``POST
/predict`` multipart field ``file`` -> detections with classifications and timing; ``GET /health``;
``GET /metrics``), but the request path never enters Python: C++ epoll threads parse HTTP, C++ decode
threads run the host half of the split JPEG decoder (csrc/runtime/jpeg_decode.h: marker parse + Huffman
decode into pinned buffers; the GPU reconstructs the frame inside the batch, csrc/kernels/jpeg_idct.hip),
the native dynamic batcher takes the upload without a copy, and C++ writes the JSON response.  Uploads the
split decoder does not cover (progressive JPEG, PNG, ...) go to the spawned PIL decode processes through
shared memory (server/decode_pool.py, native mode).  Python only builds the engines, renders Prometheus text
once a second and watches for device faults.

Run: ``python -m inference_arena_amd.server.native_front`` (PORT, ARENA_GPUS / ARENA_GPU,
ARENA_INSTANCES, ARENA_DECODE_PROCS, ARENA_HTTP_THREADS, ...) or ``ARENA_NATIVE_HTTP=1`` with the
replica launcher (parallel/replicas.py).
"""
from __future__ import annotations

import logging
import os
import signal
import threading
import time

from prometheus_client import CollectorRegistry, generate_latest
from prometheus_client.core import CounterMetricFamily, GaugeMetricFamily, HistogramMetricFamily

from ..labels import load_labels
from ..utils.logging import setup_logging
from ..utils.settings import Settings
from .decode_pool import ProcessDecodePool

log = logging.getLogger("arena.native_front")


class _Collector:
    """Prometheus families of server/metrics (arena_*) rendered from the native counters."""

    def __init__(self, front: "NativeFrontEnd", arch: str, gpu: str):
        self.front, self.arch, self.gpu = front, arch, gpu

    def collect(self):
        s = self.front.stats()
        b = self.front.batcher.stats() if self.front.batcher is not None else {"queue_depth": 0, "batch_hist": []}
        req = CounterMetricFamily("arena_requests_total", "Requests by status", labels=["arch", "status"])
        for status, key in (("ok", "ok"), ("bad_request", "bad_request"), ("too_large", "too_large"),
                            ("unavailable", "unavailable"), ("error", "errors")):
            req.add_metric([self.arch, status], s[key])
        yield req
        det = CounterMetricFamily("arena_detections_total", "Detections returned", labels=["arch"])
        det.add_metric([self.arch], s["detections"])
        yield det
        bounds = [v / 1e3 for v in s["latency_buckets_ms"]]

        def cumulative(hist):
            cum, out = 0, []
            for i, n in enumerate(hist):
                cum += n
                out.append((str(bounds[i]) if i < len(bounds) else "+Inf", cum))
            return out
        lat = HistogramMetricFamily("arena_request_latency_seconds", "Request latency by stage",
                                    labels=["arch", "stage"])
        # decode / queue / gpu / detection / classification / total (the dashboards' stage panels); the device
        # stage times come from the program's wall-clock stamps (csrc/runtime/http_front.cpp kStages)
        stages = s.get("stages") or {"total": (s["latency_hist"], s["sum_total_ms"])}
        for stage, (hist, sum_ms) in stages.items():
            lat.add_metric([self.arch, stage], cumulative(hist), sum_ms / 1e3)
        yield lat
        q = GaugeMetricFamily("arena_queue_depth", "Requests waiting in the dynamic batcher", labels=["arch", "gpu"])
        q.add_metric([self.arch, self.gpu], b["queue_depth"])
        yield q
        hist = b.get("batch_hist", [])
        cum, bb, total = 0, [], 0.0
        for size in (1, 2, 4, 8, 16, 24, 32, 48, 64):
            cum = sum(hist[:size + 1])
            bb.append((str(size), cum))
        total = float(sum(i * n for i, n in enumerate(hist)))
        bb.append(("+Inf", sum(hist)))
        bs = HistogramMetricFamily("arena_batch_size", "Executed batch sizes", labels=["arch"])
        bs.add_metric([self.arch], bb, total)
        yield bs
        oc = GaugeMetricFamily("arena_open_connections", "Open HTTP connections", labels=["arch"])
        oc.add_metric([self.arch], s["open_connections"])
        yield oc


def _http_timeouts() -> dict:
    out = {}
    for key, env in (("idle_timeout_ms", "ARENA_HTTP_IDLE_TIMEOUT_MS"), ("read_timeout_ms", "ARENA_HTTP_READ_TIMEOUT_MS")):
        if os.environ.get(env):
            out[key] = int(os.environ[env])
    return out


class NativeFrontEnd:
    """The native HTTP server over a DynamicBatcher plus its decode processes."""

    def __init__(self, batcher, labels: list[str], *, port: int = 8100, host: str = "0.0.0.0",
                 io_threads: int = 4, decode_procs: int = 2, slots: int = 512, softmax: bool = False,
                 arch: str = "monolithic", gpu: str = "0", replica_tag: str = "", decode_threads: int = 8,
                 jpeg_device: bool = True, kserve_model: str = "", **http: int):
        """``decode_threads``: native split-decoder threads (0: every upload to the ``decode_procs`` PIL
        processes, the round-3 path); ``jpeg_device=False`` reconstructs on the host threads instead of the GPU
        (instances without the device half, e.g. the host-only EchoInstance, take either).  ``http``: further
        FrontConfig fields (max_body, idle_timeout_ms, read_timeout_ms; defaults from ARENA_HTTP_IDLE_TIMEOUT_MS
        / ARENA_HTTP_READ_TIMEOUT_MS, else csrc/runtime/http_front.h)."""
        from ..ops import native
        from ..processing.transforms import max_image_pixels

        self.batcher = batcher
        self.pool = ProcessDecodePool(workers=max(1, decode_procs), slots=slots, native=True)
        self.fe = native().HttpFrontEnd(batcher, self.pool.native_channel(), list(labels),
                                        {"host": host, "port": int(port), "io_threads": int(io_threads),
                                         "softmax_confidence": bool(softmax), "replica_tag": str(replica_tag),
                                         "decode_threads": int(decode_threads), "jpeg_device": bool(jpeg_device),
                                         "max_image_pixels": int(max_image_pixels()),
                                         "kserve_model": str(kserve_model),
                                         **_http_timeouts(), **{k: int(v) for k, v in http.items()}})
        self.registry = CollectorRegistry()
        self.registry.register(_Collector(self, arch, gpu))
        self.extra_metrics = ""  # appended to /metrics (e.g. the rank's host placement, affinity.rank_info_metrics)
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._refresh, name="native-front-metrics", daemon=True)
        self._thread.start()

    @property
    def port(self) -> int:
        return self.fe.port

    def stats(self) -> dict:
        return self.fe.stats()

    def set_healthy(self, ok: bool) -> None:
        self.fe.set_healthy(bool(ok))

    def _refresh(self) -> None:
        # ARENA_MALLOC_TRIM_S (default 0 = off): return free heap pages to the kernel every that many seconds.  Round 5
        # needed it (115 MB back, tools/leak_probe_gpu.py --trim): request bodies were allocated on the I/O threads
        # and freed on the decode threads.  They now go back to the front end's body pool (csrc/runtime/
        # string_pool.h) instead of to the allocator, so no per-request buffer crosses threads.
        trim_s = float(os.environ.get("ARENA_MALLOC_TRIM_S", "0"))
        last_trim = time.monotonic()
        from ..ops import native

        while not self._stop.is_set():
            try:
                self.fe.set_metrics_text(generate_latest(self.registry).decode() + self.extra_metrics)
            except Exception as e:  # noqa: BLE001 - metrics must never stop the server
                log.warning(f"metrics refresh failed: {e}")
            if trim_s > 0 and time.monotonic() - last_trim >= trim_s:
                native().malloc_trim()
                last_trim = time.monotonic()
            self._stop.wait(1.0)

    def close(self) -> None:
        self._stop.set()
        self.fe.stop()
        self.pool.close()


def serve(settings: Settings | None = None, *, weights=None, replica_tag: str = "", devices=None) -> int:
    """Monolithic arm, native front end: engines on ``devices`` (default ARENA_GPUS / ARENA_GPU) behind one
    batcher; ``weights``: a folded weight blob (the replica launcher's broadcast).  Returns 3 after a device
    fault (the replica supervisor restarts the process), 0 on SIGTERM / SIGINT."""
    from ..engine.registry import build_session
    from ..models.zoo import resolve_models
    from ..ops import native
    from .backends import settings_devices

    from .decode_pool import prestart

    prestart()  # the decode workers' fork server, before the engines touch the GPU
    settings = settings or Settings.from_env()
    setup_logging(settings.LOG_LEVEL)
    devices = list(devices) if devices is not None else settings_devices(settings)
    instances = max(1, int(settings.ARENA_INSTANCES))
    max_batch = int(settings.ARENA_MAX_BATCH)
    fake = settings.ARENA_DEVICE == "fake"
    # host placement of this replica: its GPU's CPU share and a host thread plan sized for it (ARENA_LOCAL_WORLD
    # replicas on the node; parallel/affinity.py rank_host_setup)
    from ..parallel.affinity import rank_host_setup, rank_info_metrics

    world = int(os.environ.get("ARENA_LOCAL_WORLD", "1") or 1)
    host = rank_host_setup(devices[0] if devices else 0, world, do_pin=world > 1)
    if fake:
        # host-only stand-in for the device (CPU tests of the node layout): fixed per-replica capacity
        from .backends import fake_instance

        exs = [fake_instance(max_batch) for _ in range(instances)]
    else:
        yolo, mnet = resolve_models(settings.MODELS_DIR, int(settings.ARENA_WEIGHT_SEED))
        buckets = sorted({b for b in (1, 2, 4, 8, 16, 32, max_batch) if b <= max_batch})
        pipes = [build_session("pipeline", yolo, mnet, device=d, buckets=buckets, weights=weights) for d in devices
                 for _ in range(instances)]
        exs = [p.ex for p in pipes]
    batcher = native().DynamicBatcher(exs, {
        "max_batch": max_batch, "max_queue_delay_us": int(settings.ARENA_QUEUE_DELAY_US),
        # a lone request on an idle device is not held for the full queue delay (bench.py batcher_config; the
        # protocol's 1-user level paid 0.51 ms of queue per request without it, profiles/protocol_r5/)
        "idle_queue_delay_us": int(os.environ.get("ARENA_IDLE_QUEUE_DELAY_US", "100")),
        "max_queue_size": int(os.environ.get("ARENA_MAX_QUEUE", "4096")),
        # one process per GPU: admit due batches into free slots while older ones run (100 users: 8.4k vs 6.8k
        # req/s, profiles/r5ov/); the Triton arm's three model-server processes per GPU keep it off
        "overlap": int(os.environ.get("ARENA_BATCH_OVERLAP", "1"))})
    plan = host["plan"] if world > 1 else {"http_io": int(os.environ.get("ARENA_HTTP_THREADS", "4")),
                                           "decode_threads": int(os.environ.get("ARENA_DECODE_THREADS", "8"))}
    front = NativeFrontEnd(batcher, load_labels(settings.LABELS_FILE or None), port=int(settings.PORT),
                           io_threads=plan["http_io"],
                           # native split-decoder threads; the PIL processes only take what it does not cover
                           # (ARENA_DECODE_THREADS=0: all uploads through 10 PIL processes, the round-3 setup)
                           decode_threads=plan["decode_threads"],
                           decode_procs=int(os.environ.get("ARENA_DECODE_PROCS", "0") or
                                            (2 if plan["decode_threads"] > 0 else 10)),
                           softmax=(settings.ARENA_CONFIDENCE or "logit") == "softmax",
                           gpu=",".join(str(d) for d in devices), replica_tag=replica_tag, jpeg_device=not fake)
    front.extra_metrics = rank_info_metrics(dict(host, plan=plan), "monolithic")
    log.info("native monolithic front end ready", extra={"port": front.port, "gpus": devices,
                                                         "cpus": host["cpus"], "host_plan": plan})
    done = threading.Event()
    if threading.current_thread() is threading.main_thread():
        for sig in (signal.SIGTERM, signal.SIGINT):
            signal.signal(sig, lambda *_: done.set())
    rc = 0
    while not done.wait(0.5):
        # A batch that failed with a HIP runtime error poisons this process's device context, and a dead decode
        # worker leaves its uploads unanswered (the native front end owns its pipes): leave rotation and exit 3
        # so the replica launcher restarts the process.  Other failed batches (an input the staging pool cannot
        # take) only fail their own requests (batching.is_device_fault; reference: 500 per request).
        st = batcher.stats()
        reason = (f"device fault: {st.get('last_error', '')}" if st.get("device_faults", 0) > 0 else
                  "decode worker died" if front.pool.dead_workers > 0 else None)
        if reason:
            log.error(f"{reason}; exiting for a restart")
            front.set_healthy(False)
            front.fe.drain()  # leave the SO_REUSEPORT group; answer what is in flight
            time.sleep(1.0)
            rc = 3
            break
    front.close()
    batcher.shutdown()
    return rc


if __name__ == "__main__":
    raise SystemExit(serve())
