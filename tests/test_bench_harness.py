"""bench.py's harness on CPU: the N-rank self-launch over gloo with the host-only
fake engine, the HTTP path through the native front end and load generator, the replica weight check, and
the per-rank CPU share derived from the KFD topology."""
from __future__ import annotations

import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def _bench(*args, env=None):
    e = dict(os.environ, ARENA_DIST_BACKEND="gloo", PYTHONPATH=str(ROOT), **(env or {}))
    return subprocess.run([sys.executable, str(ROOT / "bench.py"), "--fake-engine", "--steps", "2", "--warmup", "1",
                           "--min-warmup-s", "0.3", "--users", "16", "--step-batches", "8", *args],
                          capture_output=True, text=True, timeout=600, env=e)


def test_bench_two_ranks_self_launch_http():
    r = _bench("--gpus", "2", "--latency-levels", "1,4")
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert out["n_gpus"] == 2 and out["world_size_checked"] == 2 and out["config"]["parallelism"] == "dp2"
    assert out["path"] == "http" and out["errors"] == 0 and out["value"] > 0
    assert out["weights_verified"] is True and out["collective_backend"] == "gloo"
    assert len(out["per_rank_req_s"]) == 2 and len(out["usable_cpus_per_rank"]) == 2
    assert set(out["levels"]) == {"1", "4", "batcher"} and out["bs1_p50_ms"] == out["levels"]["1"]["p50_ms"]
    assert out["inproc"]["value"] > 0 and out["inproc"]["errors"] == 0
    assert out["ms_per_step"] * out["steps"] / 1e3 == pytest.approx(2 * 256 * 2 / out["value"], rel=1e-3)
    # one node-level front door (SO_REUSEPORT, one load generator) next to the per-rank sum
    assert out["front"] == "per-rank" and out["shared_front"]["value"] > 0 and out["shared_front"]["errors"] == 0
    assert out["shared_front"]["users"] == 32 and out["mean_batch"] > 0
    # the per-request host CPU breakdown: every upload went through the native split decoder
    assert out["stage_cpu_us_per_req"]["native_decoded"] >= 2 * 256 and out["stage_cpu_us_per_req"]["fallback_decoded"] == 0
    assert out["host_cpu_us_per_req"]["total"] > 0 and out["host_cpu_us_per_req"]["decode"] > 0


def test_bench_shared_front_headline():
    r = _bench("--gpus", "2", "--front", "shared", "--latency-levels", "", "--no-secondary-inproc")
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert out["front"] == "shared" and out["errors"] == 0 and out["value"] == out["shared_front"]["value"]
    assert out["ms_per_step"] * out["steps"] / 1e3 == pytest.approx(2 * 256 * 2 / out["value"], rel=1e-3)


def test_bench_divides_the_job_cpu_quota_between_ranks():
    """4 ranks on a job quota of 8 CPUs: each rank sizes its host threads for 2 CPUs, says so loudly, and the
    node's decode processes stay within the quota."""
    r = _bench("--gpus", "4", "--latency-levels", "", "--no-secondary-inproc", "--no-secondary-shared-front",
               env={"ARENA_CPU_QUOTA": "8"})
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert out["usable_cpus_per_rank"] == [2, 2, 2, 2]
    plan = out["config"]["host_plan_per_gpu"]
    assert plan["decode_threads"] == 1 and plan["http_io"] == 1 and plan["loadgen"] == 1
    assert 4 * plan["pil_procs"] <= 8  # decode processes of the whole node within the job quota
    assert out["cpu_budget_warning"] and "only 2 usable CPUs" in r.stderr
    assert out["errors"] == 0 and out["value"] > 0
    # one physical device per rank, recorded
    assert out["torch_world_size"] == 4 and out["distinct_gpus"] == 4 and not out["shared_gpu_rehearsal"]
    assert [d["rank"] for d in out["rank_devices"]] == [0, 1, 2, 3]
    assert len({d["pci_bus_id"] for d in out["rank_devices"]}) == 4


def test_bench_refuses_two_ranks_on_one_gpu():
    r = _bench("--gpus", "2", "--latency-levels", "", "--no-secondary-inproc", "--no-secondary-shared-front",
               env={"ARENA_TEST_DUP_BUS": "1"})
    assert r.returncode != 0 and "drive the same GPU" in r.stderr
    r = _bench("--gpus", "2", "--latency-levels", "", "--no-secondary-inproc", "--no-secondary-shared-front",
               env={"ARENA_TEST_DUP_BUS": "1", "ARENA_SHARED_GPU": "1"})
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert out["shared_gpu_rehearsal"] is True and out["distinct_gpus"] == 1


def test_bench_detects_diverging_replica_weights():
    r = _bench("--gpus", "2", "--latency-levels", "", "--no-secondary-inproc", env={"ARENA_TEST_CORRUPT_WEIGHTS": "1"})
    assert r.returncode != 0
    assert "replica weights differ" in r.stderr


def _fake_topology(tmp: Path, gpus_numa: list[int], cpus_per_numa: int = 8):
    nodes = tmp / "nodes"
    pci = tmp / "pci"
    (nodes / "0").mkdir(parents=True)
    (nodes / "0" / "properties").write_text("cpu_cores_count 64\nsimd_count 0\n")  # the CPU node
    for g, numa in enumerate(gpus_numa):
        n = nodes / str(g + 1)
        n.mkdir()
        bus = 0x10 + g
        (n / "properties").write_text(f"simd_count 1024\nlocation_id {bus << 8}\ndomain 0\n")
        d = pci / f"0000:{bus:02x}:00.0"
        d.mkdir(parents=True)
        lo = numa * cpus_per_numa
        (d / "local_cpulist").write_text(f"{lo}-{lo + cpus_per_numa - 1}\n")
        (d / "numa_node").write_text(f"{numa}\n")
    return nodes, pci


def test_rank_cpu_share_splits_numa_nodes(tmp_path, monkeypatch):
    from inference_arena_amd.parallel import affinity

    nodes, pci = _fake_topology(tmp_path, [0, 0, 1, 1])
    monkeypatch.setattr(affinity.os, "sched_getaffinity", lambda pid: set(range(16)), raising=False)
    monkeypatch.delenv("HIP_VISIBLE_DEVICES", raising=False)
    monkeypatch.delenv("ROCR_VISIBLE_DEVICES", raising=False)
    shares = [affinity.rank_cpu_share(r, 4, nodes, pci) for r in range(4)]
    assert shares == [[0, 1, 2, 3], [4, 5, 6, 7], [8, 9, 10, 11], [12, 13, 14, 15]]
    assert affinity.gpu_local_cpus(2, nodes, pci) == (list(range(8, 16)), 1)
    assert affinity.rank_cpu_share(0, 1, tmp_path / "missing", pci) is None
