"""RQ2 / RQ3 analyses (CPU): cost model, LOC counting, per-arm complexity, resource sampler."""
from __future__ import annotations

import math
import os
import time

import pytest

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


def test_cost_config_validates():
    from inference_arena_amd.config import get_cost_config, validate_config

    c = get_cost_config()
    assert c["gpu_hour_usd"] > 0 and c["vcpu_hour_usd"] >= 0
    assert validate_config() == []
