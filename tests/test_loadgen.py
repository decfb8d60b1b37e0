"""Load generator against a live uvicorn monolithic service (fake backend, CPU)."""
from __future__ import annotations

import socket
import threading
import time

import numpy as np

from inference_arena_amd.data.synthetic import encode_jpeg, synthetic_images
from inference_arena_amd.loadgen.hypotheses import evaluate
from inference_arena_amd.loadgen.runner import LoadConfig, run_level, summarize, write_level


def _serve(app):
    import uvicorn

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    server = uvicorn.Server(uvicorn.Config(app, host="127.0.0.1", port=port, log_level="error"))
    t = threading.Thread(target=server.run, daemon=True)
    t.start()
    for _ in range(100):
        if server.started:
            break
        time.sleep(0.05)
    return server, t, port


def test_closed_loop_against_live_server(tmp_path):
    from tests.test_server_monolithic import FakeBackend

    from inference_arena_amd.server.monolithic import create_app
    from inference_arena_amd.utils.settings import Settings

    app = create_app(Settings(LOG_LEVEL="WARNING", ARENA_FAULT_EVERY=10), FakeBackend())
    server, t, port = _serve(app)
    try:
        imgs = [encode_jpeg(im) for im in synthetic_images(3, 1, hw=(120, 160))]
        cfg = LoadConfig(url=f"http://127.0.0.1:{port}/predict", users=3, warmup_s=0.3, measure_s=1.0,
                         cooldown_s=0.2)
        res = run_level(cfg, imgs)
        s = summarize(res, cfg)
        write_level(tmp_path, "mono_u3", res, s)
    finally:
        server.should_exit = True
        t.join(10)
    assert s["requests"] > 10 and s["throughput_rps"] > 5
    assert 5 <= s["error_rate_percent"] <= 15  # every 10th request fails (fault injection)
    assert s["p50_latency_ms"] <= s["p99_latency_ms"]
    assert s["mean_detections"] == 2
    assert (tmp_path / "mono_u3_stats.csv").read_text().startswith("Type,Name,Request Count")
    assert {r[1] for r in res.samples} == {0, 1, 2}


def test_native_engine_closed_loop(tmp_path):
    """ARENA_LOADGEN=native: the same closed loop from the C++ load generator (csrc/runtime/http_loadgen.cpp) —
    requests counted in the window, the injected failures as errors, detections parsed from the JSON."""
    from tests.test_server_monolithic import FakeBackend

    from inference_arena_amd.server.monolithic import create_app
    from inference_arena_amd.utils.settings import Settings

    app = create_app(Settings(LOG_LEVEL="WARNING", ARENA_FAULT_EVERY=10), FakeBackend())
    server, t, port = _serve(app)
    try:
        imgs = [encode_jpeg(im) for im in synthetic_images(3, 1, hw=(120, 160))]
        cfg = LoadConfig(url=f"http://127.0.0.1:{port}/predict", users=3, warmup_s=0.3, measure_s=1.0,
                         cooldown_s=0.2, procs=2, engine="native")
        res = run_level(cfg, imgs)
        s = summarize(res, cfg)
    finally:
        server.should_exit = True
        t.join(10)
    assert s["loadgen"] == "native" and s["requests"] > 10 and s["throughput_rps"] > 5
    assert 5 <= s["error_rate_percent"] <= 15
    assert s["p50_latency_ms"] <= s["p99_latency_ms"] and s["mean_detections"] == 2


def test_hypothesis_evaluation():
    rows = []
    for arch, p99, p50 in (("monolithic", 10, 5), ("microservices", 11, 6), ("triton", 12, 5)):
        for u in (1, 10, 50, 75):
            rows.append({"architecture": arch, "users": u, "p99_latency_ms": p99 * u, "p50_latency_ms": p50 * u,
                         "throughput_rps": 100.0, "error_rate_percent": 0.0})
    r = evaluate(rows)
    assert r["H1a"]["supported"] and r["H1b"]["supported"]
    assert not r["H1c"]["supported"]  # triton gap 7u > micro gap 5u
    assert r["H1d"]["saturation_users"]["monolithic"] == 75
    assert np.isclose(r["H1b"]["overhead"][10], 0.1)
