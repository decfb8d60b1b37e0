"""Closed-loop HTTP load generator for the three topologies.

Semantics follow the reference's experiment spec (experiment.yaml
``load_testing``): N concurrent users, each sending
``POST /predict`` (multipart ``file``) and immediately the next request when
the response arrives (no think time), with warmup / measurement / cooldown
phases and several runs per (architecture, users) configuration.  Only
requests *completed* inside the measurement window count.

Outputs per level: a per-request CSV (t, user, latency_ms, status,
detections), a Locust-compatible ``*_stats.csv`` row set, and a summary
(p50/p90/p95/p99 latency, throughput_rps, error_rate_percent) — the metrics
experiment.yaml lists for the hypotheses.

Many users need many sockets: the generator runs one aiohttp session per
process and can fan out over ``procs`` processes (multiprocessing) so that
the client is never the bottleneck at high load.  ``engine="native"``
(``ARENA_LOADGEN=native``) drives the same closed loop from the C++ epoll
load generator (csrc/runtime/http_loadgen.cpp, ``procs`` threads): at
thousands of requests/s the Python client's own CPU competes with the servers
on a shared box.
"""
from __future__ import annotations

import asyncio
import csv
import json
import os
import multiprocessing as mp
import random
import time
from dataclasses import asdict, dataclass, field
from dataclasses import field as dc_field
from pathlib import Path

import numpy as np


@dataclass
class LoadConfig:
    url: str = "http://127.0.0.1:8100/predict"
    users: int = 1
    warmup_s: float = 60.0
    measure_s: float = 180.0
    cooldown_s: float = 30.0
    timeout_s: float = 30.0
    procs: int = 1
    seed: int = 42
    field: str = "file"
    engine: str = dc_field(default_factory=lambda: os.environ.get("ARENA_LOADGEN", "aiohttp"))


@dataclass
class PhaseResult:
    users: int
    samples: list = field(default_factory=list)  # (t_end_rel, user, latency_ms, status, detections)
    wall_s: float = 0.0


def _bodies(images: list[bytes], fieldname: str) -> list[tuple[bytes, str]]:
    """Pre-encoded multipart bodies: one buffer per request, no per-request form building."""
    from ..server.multipart import encode_multipart

    return [encode_multipart(fieldname, img, "image.jpg") for img in images]


async def _user_loop(session, cfg: LoadConfig, uid: int, bodies: list[tuple[bytes, str]], t_start: float,
                     t_stop: float, out: list) -> None:
    import aiohttp

    rng = random.Random(cfg.seed * 1000 + uid)
    while time.perf_counter() < t_stop:
        body, ctype = bodies[rng.randrange(len(bodies))]
        t0 = time.perf_counter()
        status, ndet = 0, -1
        try:
            async with session.post(cfg.url, data=body, headers={"content-type": ctype}) as r:
                body = await r.read()
                status = r.status
                if status == 200:
                    try:
                        ndet = len(json.loads(body)["detections"])
                    except (ValueError, KeyError):
                        ndet = -1
        except (aiohttp.ClientError, asyncio.TimeoutError):
            status = 599
        t1 = time.perf_counter()
        out.append((t1 - t_start, uid, (t1 - t0) * 1e3, status, ndet))


async def _drive(cfg: LoadConfig, users: range, images: list[bytes]) -> list:
    import aiohttp

    total = cfg.warmup_s + cfg.measure_s + cfg.cooldown_s
    conn = aiohttp.TCPConnector(limit=0, force_close=False)
    timeout = aiohttp.ClientTimeout(total=cfg.timeout_s)
    out: list = []
    bodies = _bodies(images, cfg.field)
    async with aiohttp.ClientSession(connector=conn, timeout=timeout) as s:
        t_start = time.perf_counter()
        await asyncio.gather(*(_user_loop(s, cfg, u, bodies, t_start, t_start + total, out) for u in users))
    return out


def _proc_main(args):
    cfg, users, images = args
    return asyncio.run(_drive(cfg, users, images))


def _run_native(cfg: LoadConfig, images: list[bytes]) -> list:
    """The closed loop on the C++ load generator: every user keeps one keep-alive connection busy for the three
    phases; samples carry user -1 (the generator does not tag requests by user)."""
    from urllib.parse import urlsplit

    from ..ops import native
    from ..server.multipart import encode_multipart

    u = urlsplit(cfg.url)
    reqs = []
    for img in images:
        body, ctype = encode_multipart(cfg.field, img, filename="image.jpg", content_type="image/jpeg")
        reqs.append((f"POST {u.path or '/'} HTTP/1.1\r\nHost: {u.hostname}\r\nContent-Type: {ctype}\r\n"
                     f"Content-Length: {len(body)}\r\n\r\n").encode() + body)
    random.Random(cfg.seed).shuffle(reqs)
    lg = native().HttpLoadGen({"host": u.hostname or "127.0.0.1", "port": u.port or 80, "users": cfg.users,
                               "threads": max(1, min(cfg.procs, cfg.users))}, reqs)
    lg.start()
    time.sleep(cfg.warmup_s + cfg.measure_s + cfg.cooldown_s)
    lg.stop(cfg.timeout_s)
    r = lg.records()
    return [(float(t), -1, float(lat) * 1e3, int(st) if st > 0 else 599, int(d))
            for t, lat, st, d in zip(r["t_done"], r["latency"], r["status"], r["dets"])]


def _heartbeat(cfg: LoadConfig, stop) -> None:
    """A progress line every 30 s: a level at the reference's length (60 + 180 + 30 s) is otherwise silent for
    minutes, which supervisors of batch jobs read as a hang."""
    import threading

    def run():
        t0 = time.perf_counter()
        total = cfg.warmup_s + cfg.measure_s + cfg.cooldown_s
        while not stop.wait(30.0):
            print(f"[loadgen] users={cfg.users}: {time.perf_counter() - t0:.0f} / {total:.0f} s", flush=True)

    threading.Thread(target=run, daemon=True, name="loadgen-heartbeat").start()


def run_level(cfg: LoadConfig, images: list[bytes]) -> PhaseResult:
    """Run one (users) level with all phases; returns every completed request."""
    import threading

    stop = threading.Event()
    _heartbeat(cfg, stop)
    try:
        return _run_level(cfg, images)
    finally:
        stop.set()


def _run_level(cfg: LoadConfig, images: list[bytes]) -> PhaseResult:
    t0 = time.perf_counter()
    if cfg.engine == "native":
        return PhaseResult(cfg.users, sorted(_run_native(cfg, images)), time.perf_counter() - t0)
    procs = max(1, min(cfg.procs, cfg.users))
    if procs == 1:
        samples = asyncio.run(_drive(cfg, range(cfg.users), images))
    else:
        chunks = [range(i, cfg.users, procs) for i in range(procs)]
        with mp.get_context("spawn").Pool(procs) as pool:
            parts = pool.map(_proc_main, [(cfg, c, images) for c in chunks])
        samples = [s for p in parts for s in p]
    return PhaseResult(cfg.users, sorted(samples), time.perf_counter() - t0)


def summarize(res: PhaseResult, cfg: LoadConfig) -> dict:
    lo, hi = cfg.warmup_s, cfg.warmup_s + cfg.measure_s
    win = [s for s in res.samples if lo <= s[0] < hi]
    lat = np.array([s[2] for s in win if s[3] == 200], dtype=np.float64)
    n_err = sum(1 for s in win if s[3] != 200)
    n = len(win)
    q = (lambda p: float(np.percentile(lat, p)) if lat.size else float("nan"))  # noqa: E731
    ndet = [s[4] for s in win if s[3] == 200 and s[4] >= 0]
    return {
        "users": res.users,
        "requests": n,
        "failures": n_err,
        "throughput_rps": (n - n_err) / cfg.measure_s if cfg.measure_s > 0 else float("nan"),
        "error_rate_percent": 100.0 * n_err / n if n else 0.0,
        "p50_latency_ms": q(50), "p90_latency_ms": q(90), "p95_latency_ms": q(95), "p99_latency_ms": q(99),
        "mean_latency_ms": float(lat.mean()) if lat.size else float("nan"),
        "max_latency_ms": float(lat.max()) if lat.size else float("nan"),
        "mean_detections": float(np.mean(ndet)) if ndet else float("nan"),
        "measure_s": cfg.measure_s,
        "loadgen": cfg.engine,
    }


def write_level(out_dir: Path, tag: str, res: PhaseResult, summary: dict) -> None:
    out_dir.mkdir(parents=True, exist_ok=True)
    with open(out_dir / f"{tag}_requests.csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["t_s", "user", "latency_ms", "status", "detections"])
        w.writerows(res.samples)
    # Locust-compatible aggregate (the spec'd tool's stats layout)
    with open(out_dir / f"{tag}_stats.csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Type", "Name", "Request Count", "Failure Count", "Median Response Time",
                    "Average Response Time", "Max Response Time", "Requests/s", "95%", "99%"])
        w.writerow(["POST", "/predict", summary["requests"], summary["failures"], summary["p50_latency_ms"],
                    summary["mean_latency_ms"], summary["max_latency_ms"], summary["throughput_rps"],
                    summary["p95_latency_ms"], summary["p99_latency_ms"]])
    # the serving configuration the level ran against (transport, fan-out, process layout, envelope ...)
    summary = dict(summary, env={k: v for k, v in sorted(os.environ.items())
                                 if k.startswith("ARENA_") or k in ("CONTAINER_VCPU", "LOG_LEVEL")})
    (out_dir / f"{tag}_summary.json").write_text(json.dumps(summary, indent=2) + "\n")


def run_sweep(base: LoadConfig, user_levels: list[int], runs: int, images: list[bytes], out_dir: Path,
              arch: str, log=print, sample_pids: list[int] | None = None, scrape: list[str] | None = None) -> list[dict]:
    """``sample_pids``: server processes (children included) whose CPU % / memory (and GPU busy / VRAM) are
    sampled during each level (loadgen/resources.py; experiment.yaml RQ2 metrics).  ``scrape``: Prometheus URLs
    (the arm's /metrics: per-stage latency histograms of the servers themselves) saved after every level."""
    rows = []
    for users in user_levels:
        for run in range(1, runs + 1):
            cfg = LoadConfig(**{**asdict(base), "users": users, "seed": base.seed + run})
            sampler = None
            if sample_pids:
                from .resources import ResourceSampler

                sampler = ResourceSampler(sample_pids).start()
            res = run_level(cfg, images)
            s = summarize(res, cfg)
            if sampler is not None:
                s.update(sampler.stop())
            s.update({"architecture": arch, "run": run})
            write_level(out_dir, f"{arch}_u{users}_r{run}", res, s)
            for i, url in enumerate(scrape or []):
                try:
                    import urllib.request

                    with urllib.request.urlopen(url, timeout=5) as r:
                        (out_dir / f"{arch}_u{users}_r{run}_metrics{i}.txt").write_bytes(r.read())
                except Exception as e:  # noqa: BLE001 - diagnostics only
                    log(f"[{arch}] scrape {url} failed: {e}")
            rows.append(s)
            log(f"[{arch}] users={users} run={run}: {s['throughput_rps']:.1f} req/s "
                f"p50={s['p50_latency_ms']:.1f} ms p99={s['p99_latency_ms']:.1f} ms err={s['error_rate_percent']:.2f}%")
    with open(out_dir / f"{arch}_sweep.csv", "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(rows[0]))
        w.writeheader()
        w.writerows(rows)
    return rows
