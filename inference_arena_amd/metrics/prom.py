"""Per-service Prometheus metrics (``GET /metrics``).

The reference installs prometheus-client but never exposes application
metrics: its Prometheus only scrapes cAdvisor container CPU/memory
(infrastructure/prometheus/prometheus.yml:57-92; the app job at :103-115 is
commented out).  Every arena service exports:

  arena_request_latency_seconds{arch,stage}  histogram (stage: total, detection,
                                             classification, queue, gpu, decode)
  arena_requests_total{arch,status}           counter
  arena_detections_total{arch}                counter
  arena_batch_size{arch}                      histogram of executed batch sizes
  arena_queue_depth{arch,gpu}                 gauge (dynamic batcher queue)
  arena_gpu_busy_ratio{arch,gpu}              gauge (GPU time / wall time, last window)
  arena_hbm_used_bytes{gpu}                   gauge (device memory in use)
and, on the model server, KServe/Triton-compatible ``nv_inference_*`` counters.
"""
from __future__ import annotations

import time

from prometheus_client import CollectorRegistry, Counter, Gauge, Histogram, generate_latest

LAT_BUCKETS = (0.0005, 0.001, 0.002, 0.005, 0.01, 0.02, 0.05, 0.1, 0.2, 0.5, 1.0, 2.0, 5.0)
BATCH_BUCKETS = (1, 2, 4, 8, 16, 24, 32, 48, 64)


class ArenaMetrics:
    def __init__(self, arch: str, gpu: str = "0", registry: CollectorRegistry | None = None):
        self.arch = arch
        self.gpu = str(gpu)
        self.registry = registry or CollectorRegistry()
        r = self.registry
        self.latency = Histogram("arena_request_latency_seconds", "Request latency by stage", ["arch", "stage"],
                                 buckets=LAT_BUCKETS, registry=r)
        self.requests = Counter("arena_requests_total", "Requests by status", ["arch", "status"], registry=r)
        self.detections = Counter("arena_detections_total", "Detections returned", ["arch"], registry=r)
        self.batch = Histogram("arena_batch_size", "Executed batch sizes", ["arch"], buckets=BATCH_BUCKETS,
                               registry=r)
        self.queue = Gauge("arena_queue_depth", "Requests waiting in the dynamic batcher", ["arch", "gpu"],
                           registry=r)
        self.busy = Gauge("arena_gpu_busy_ratio", "GPU busy fraction over the last window", ["arch", "gpu"],
                          registry=r)
        self.hbm = Gauge("arena_hbm_used_bytes", "Device memory in use", ["gpu"], registry=r)
        self._gpu_s = 0.0
        self._t = time.monotonic()

    def observe(self, status: str, timing_ms: dict | None = None, detections: int = 0, batch: int | None = None):
        self.requests.labels(self.arch, status).inc()
        if detections:
            self.detections.labels(self.arch).inc(detections)
        for k, v in (timing_ms or {}).items():
            if k.endswith("_ms"):
                self.latency.labels(self.arch, k[:-3]).observe(float(v) / 1e3)
        if batch:
            self.batch.labels(self.arch).observe(batch)

    def gpu_time(self, seconds: float) -> None:
        self._gpu_s += seconds
        now = time.monotonic()
        if now - self._t >= 1.0:
            self.busy.labels(self.arch, self.gpu).set(min(1.0, self._gpu_s / (now - self._t)))
            self._gpu_s, self._t = 0.0, now

    def render(self) -> bytes:
        return generate_latest(self.registry)
