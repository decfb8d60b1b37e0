"""RQ2 / RQ3 analyses (CPU): cost model, LOC counting, per-arm complexity, resource sampler."""
from __future__ import annotations

import math
import os
import time

import pytest
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]

from inference_arena_amd.analysis.rq import complexity_report, cost_per_1000_requests, count_loc, enrich_sweep_rows


def test_cost_per_1000_requests():
    # 1 GPU at 6 USD/h + 2 vCPUs at 0.04 USD/h serving 1000 req/s: (6.08 / 3600) / 1000 * 1000
    got = cost_per_1000_requests(1000.0, gpus=1, gpu_hour_usd=6.0, vcpus=2, vcpu_hour_usd=0.04)
    assert got == pytest.approx(6.08 / 3600.0)
    assert math.isnan(cost_per_1000_requests(0.0, gpus=1, gpu_hour_usd=6.0))
    rows = enrich_sweep_rows([{"throughput_rps": 500.0, "cpu_utilization_percent": 150.0}], gpus=2,
                             cost={"gpu_hour_usd": 6.0, "vcpu_hour_usd": 0.04})
    assert rows[0]["cost_per_1000_requests_usd"] == pytest.approx((12.0 + 1.5 * 0.04) / 3600.0 / 500.0 * 1000.0)


def test_count_loc_skips_comments(tmp_path):
    py = tmp_path / "a.py"
    py.write_text("# c\n\nx = 1\n  # indented comment\ny = 2  # trailing\n")
    cpp = tmp_path / "a.cpp"
    cpp.write_text("// c\n/* block\n still */\nint x;\n/* one line */\nint y; // t\n")
    assert count_loc(py) == 2 and count_loc(cpp) == 2


def test_complexity_report_covers_the_three_arms():
    r = complexity_report()
    for arm in ("monolithic", "microservices", "triton"):
        assert r[arm]["application_code_loc"] > 100 and r[arm]["configuration_loc"] > 10
    assert r["shared_engine_loc"] > 5000


def test_resource_sampler_follows_a_process_tree():
    """A busy child process (not the root) shows up in the CPU reading: children are followed and their CPU
    counters kept from sample to sample."""
    import subprocess
    import sys

    from inference_arena_amd.loadgen.resources import ResourceSampler

    child = subprocess.Popen([sys.executable, "-c", "import time\nt=time.time()\nwhile time.time()-t<3: pass"])
    try:
        s = ResourceSampler([os.getpid()], interval=0.2, gpu=False).start()
        time.sleep(1.5)
        out = s.stop()
    finally:
        child.kill()
        child.wait()
    assert out["resource_samples"] >= 4
    assert out["memory_usage_mb"] > 10
    assert out["cpu_utilization_percent_max"] > 50.0, out  # the spinning child: ~100 % of one core
    # RSS per role: the roles' last samples add up to about the total
    by = out["memory_mb_by_role"]
    assert by and all(v["mean"] > 0 and v["last"] > 0 for v in by.values()), by
    assert abs(sum(v["mean"] for v in by.values()) - out["memory_usage_mb"]) < 0.05 * out["memory_usage_mb"] + 5


def test_resource_sampler_splits_cpu_by_thread_class():
    """cpu_percent_by_thread: a named busy thread (prctl PR_SET_NAME, as the native threads name themselves) is
    reported under its class, its trailing index dropped."""
    import ctypes
    import hashlib
    import threading

    from inference_arena_amd.loadgen.resources import ResourceSampler

    assert ResourceSampler.thread_class("arena-jpeg3") == "arena-jpeg"
    assert ResourceSampler.thread_class("python3") == "python"
    stop = threading.Event()
    blob = bytes(1 << 22)

    def spin():  # busy in C with the GIL released (hashlib drops it for large inputs): no GIL convoy
        ctypes.CDLL(None).prctl(15, b"arena-spin7", 0, 0, 0)  # PR_SET_NAME
        while not stop.is_set():
            hashlib.sha256(blob).digest()

    t = threading.Thread(target=spin, daemon=True)
    t.start()
    try:
        s = ResourceSampler([os.getpid()], interval=0.2, gpu=False).start()
        time.sleep(1.5)
        out = s.stop()
    finally:
        stop.set()
        t.join()
    by = out.get("cpu_percent_by_thread", {})
    spin_pct = sum(v.get("arena-spin", 0.0) for v in by.values())
    assert spin_pct > 20.0, (out, s.by_thread)


def test_cost_config_validates():
    from inference_arena_amd.config import get_cost_config, validate_config

    c = get_cost_config()
    assert c["gpu_hour_usd"] > 0 and c["vcpu_hour_usd"] >= 0
    assert validate_config() == []


def _rows():
    """Synthetic sweep rows: monolithic fastest at low load, triton catching up past ~60 users on throughput."""
    out = []
    spec = {
        "monolithic": {1: (300, 2.5, 3.0, 120, 3000), 10: (2800, 3.5, 4.0, 350, 3100),
                       50: (5400, 9.0, 10.0, 500, 3200), 100: (6000, 15.0, 17.0, 600, 3300)},
        "microservices": {1: (150, 6.0, 9.0, 160, 5000), 10: (950, 10.0, 17.0, 900, 5100),
                          50: (1600, 27.0, 120.0, 1300, 5200), 100: (1700, 50.0, 200.0, 1300, 5300)},
        "triton": {1: (280, 2.7, 3.5, 150, 6000), 10: (1300, 7.0, 13.0, 400, 6100),
                   50: (4900, 10.0, 16.0, 1000, 6200), 100: (6500, 15.0, 28.0, 1100, 6300)},
    }
    for arch, lv in spec.items():
        for u, (rps, p50, p99, cpu, mem) in lv.items():
            for run in (1, 2):
                out.append({"architecture": arch, "users": u, "run": run, "throughput_rps": rps + run,
                            "p50_latency_ms": p50, "p99_latency_ms": p99, "cpu_utilization_percent": cpu,
                            "memory_usage_mb": mem, "error_rate_percent": 0.0,
                            "cost_per_1000_requests_usd": 1.0 / rps})
    return out


def test_h2_h3_and_rq4_from_sweep_rows():
    from inference_arena_amd.analysis.decision import analyze

    rq3 = {"monolithic": {"application_code_loc": 2000, "configuration_loc": 50},
           "microservices": {"application_code_loc": 1100, "configuration_loc": 80},
           "triton": {"application_code_loc": 1300, "configuration_loc": 70}}
    deploy = {"monolithic": {"deployment_time_seconds": 8.0, "runs": [8, 8, 8], "baseline_memory_mb": 2900},
              "microservices": {"deployment_time_seconds": 12.0, "runs": [12] * 3, "baseline_memory_mb": 5000},
              "triton": {"deployment_time_seconds": 15.0, "runs": [15] * 3, "baseline_memory_mb": 6000}}
    out = analyze(_rows(), rq3, deploy)
    h = out["hypotheses"]
    assert h["H2a"]["supported"] and h["H2a"]["supported_configured"]  # 2 vs 4 vCPU in deploy/compose
    assert h["H2b"]["supported"]
    assert h["H2c"]["supported"] and h["H2c"]["source"]["triton"] == "idle after ready"
    assert h["H2d"]["levels"] == [50, 100] and "supported" in h["H2d"]
    assert h["H3a"]["supported"]  # 1300 < 2000 application LOC
    assert h["H3b"]["supported"] and h["H3c"]["supported"]
    # throughput: triton overtakes monolithic between 50 and 100 users
    cx = [c for c in out["rq4"]["crossover_points"] if c["pair"] == ["monolithic", "triton"]
          and c["metric"] == "throughput_rps"]
    assert len(cx) == 1 and 50 < cx[0]["users"] < 100
    assert cx[0]["better_below"] == "monolithic" and cx[0]["better_above"] == "triton"
    dm = out["rq4"]["decision_matrix"]
    assert dm["by_load_regime"]["low (<= 10 users)"]["lowest_p99_ms"]["best"] == "monolithic"
    assert dm["by_load_regime"]["high (>= 75 users)"]["highest_throughput_rps"]["best"] == "triton"
    assert dm["by_p99_slo"]["p99 <= 5 ms"]["best"] == "monolithic"
    assert dm["by_p99_slo"]["p99 <= 50 ms"]["best"] == "triton"


def test_deploy_time_with_a_fake_launcher(tmp_path):
    import subprocess
    import sys
    from pathlib import Path

    sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "scripts"))
    import deploy_time

    started = []

    def start(arch, gpus, log_dir):
        time.sleep(0.05)
        p = subprocess.Popen([sys.executable, "-c", "import time; x = bytearray(20 << 20); time.sleep(30)"])
        started.append(p)
        time.sleep(0.5)
        return [p], True

    def stop(procs):
        for p in procs:
            p.kill()
            p.wait()

    r = deploy_time.measure("monolithic", 2, 1, tmp_path, start=start, stop=stop, settle_s=0.1)
    assert len(r["runs"]) == 2 and all(0.5 <= t < 5 for t in r["runs"])
    assert r["baseline_memory_mb"] > 15  # the child's 20 MiB buffer is resident
    assert all(p.poll() is not None for p in started)


def test_analyze_results_script_with_deploy_times(tmp_path):
    """scripts/analyze_results.py end to end on sweep CSVs split over several files (one per call of a sweep) plus
    a scripts/deploy_time.py JSON: H1-H3, the deployment-time table and the RQ4 decision matrix are written."""
    import csv
    import importlib.util
    import json

    rows = _rows()
    files = []
    for i, part in enumerate((rows[: len(rows) // 2], rows[len(rows) // 2:])):
        f = tmp_path / f"sweep_{i}.csv"
        with open(f, "w", newline="") as fh:
            w = csv.DictWriter(fh, fieldnames=list(part[0]))
            w.writeheader()
            w.writerows(part)
        files.append(str(f))
    deploy = {a: {"deployment_time_seconds": t, "runs": [t, t, t], "baseline_memory_mb": m, "gpus": 1}
              for a, t, m in (("monolithic", 2.7, 2100.0), ("microservices", 3.5, 4500.0), ("triton", 5.0, 4000.0))}
    (tmp_path / "deploy.json").write_text(json.dumps(deploy))
    spec = importlib.util.spec_from_file_location("analyze_results", ROOT / "scripts" / "analyze_results.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    out = tmp_path / "analysis"
    assert mod.main([*files, "--deploy", str(tmp_path / "deploy.json"), "--gpus", "1", "--out", str(out)]) == 0
    text = (out / "summary.md").read_text()
    assert "deployment time s" in text and "| triton | 5.00 |" in text
    assert "H3c" in text and "H1a" in text and "RQ4 crossover points" in text
    summary = json.loads((out / "summary.json").read_text())
    assert summary["rq3"]["triton"]["deployment_time_seconds"] == 5.0
