"""Node-scale process layouts on CPU: ``scripts/start_arena.py`` at N = 1 and N = 4 fake GPUs.

A fake GPU (``ARENA_DEVICE=fake``, server/backends.py ``fake_instance``) answers a batch of 4 after 40 ms with
2 batches in flight, so one GPU's worth of engine serves at most 200 requests/s whatever the host does.  An arm
whose host layout scales with N (one model server + one gateway per GPU for Triton, one replica per GPU for
monolithic) then reaches about N x its N = 1 rate; a layout with one process for all GPUs (round 5's Triton arm)
stays near one GPU's host plan.  Every rank reports its CPU share and thread plan on its /metrics."""
from __future__ import annotations

import importlib.util
import io
import os
import sys
import time
import urllib.request
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

USERS_PER_GPU = 24
WINDOW_S = 4.0


def _start_arena():
    spec = importlib.util.spec_from_file_location("start_arena", ROOT / "scripts" / "start_arena.py")
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _uploads(n: int = 8) -> list[bytes]:
    from PIL import Image

    bench = _bench_module()
    rng = np.random.default_rng(3)
    out = []
    for i in range(n):
        b = io.BytesIO()
        Image.fromarray((rng.random((48, 64, 3)) * 255).astype(np.uint8)).save(b, format="JPEG", quality=90)
        out.append(bench.http_request(b.getvalue()))
    return out


def _bench_module():
    spec = importlib.util.spec_from_file_location("bench_mod", ROOT / "bench.py")
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _rate(port: int, users: int) -> tuple[float, int]:
    """Closed-loop req/s over WINDOW_S after a 1 s warm-up, and the non-200 count."""
    from inference_arena_amd.ops import native

    lg = native().HttpLoadGen({"host": "127.0.0.1", "port": port, "users": users, "threads": 2}, _uploads())
    lg.start()
    try:
        time.sleep(1.0)
        n0, t0 = lg.completed(), time.perf_counter()
        time.sleep(WINDOW_S)
        n1, t1 = lg.completed(), time.perf_counter()
    finally:
        lg.stop(30.0)
    rec = lg.records(n0, n1)
    return (n1 - n0) / (t1 - t0), int((rec["status"] != 200).sum())


def _metrics(port: int) -> str:
    with urllib.request.urlopen(f"http://127.0.0.1:{port}/metrics", timeout=5) as r:
        return r.read().decode()


@pytest.fixture(scope="module")
def repo(tmp_path_factory):
    from inference_arena_amd.repository import store

    root = tmp_path_factory.mktemp("model_repository")
    store.build_repository(root, seed=0)
    return root


def _env():
    # fake engines; the job's CPUs split between the ranks as on the GPU box (8 here for the whole node)
    return {"ARENA_FAKE_LATENCY_US": "40000", "ARENA_FAKE_SLOTS": "2", "ARENA_FAKE_MAX_BATCH": "4",
            "ARENA_MAX_BATCH": "4", "ARENA_QUEUE_DELAY_US": "2000", "ARENA_NATIVE_HTTP": "1",
            "ARENA_CPU_QUOTA": str(os.cpu_count() or 8), "ARENA_DIST_BACKEND": "gloo",
            "ARENA_DECODE_PROCS": "1"}


def _run(arch: str, gpus: int, repo: Path, tmp: Path) -> tuple[float, int, list[str]]:
    sa = _start_arena()
    old = {k: os.environ.get(k) for k in _env()}
    os.environ.update(_env())
    procs, ok = [], False
    try:
        procs, ok = sa.start(arch, gpus, tmp / f"logs_{arch}_{gpus}", device="fake", repo=str(repo))
        assert ok, f"{arch} x{gpus} did not come up: " + "".join(
            (p.read_text()[-1500:] for p in (tmp / f"logs_{arch}_{gpus}").glob("*.log")))
        port = 8100 if arch == "monolithic" else 8300
        rate, errors = _rate(port, USERS_PER_GPU * gpus)
        if arch == "triton":
            texts = [_metrics(p) for _, _, p in sa.plan_triton(gpus)["model_servers"]]
        else:
            texts = [_metrics(8100)]
        return rate, errors, texts
    finally:
        sa.stop(procs)
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def test_plan_triton_ports():
    sa = _start_arena()
    p = sa.plan_triton(4, base_port=9004)
    assert [x[2] for x in p["model_servers"]] == [9004, 9014, 9024, 9034]
    assert p["upstreams"].split(",")[3] == "127.0.0.1:9034"
    assert len(sa.plan_triton(2, 2, base_port=9004)["model_servers"]) == 4


@pytest.mark.parametrize("arch", ["triton", "monolithic"])
def test_four_fake_gpus_scale_with_the_host_layout(arch, repo, tmp_path):
    r1, e1, _ = _run(arch, 1, repo, tmp_path)
    r4, e4, texts = _run(arch, 4, repo, tmp_path)
    assert e1 == 0 and e4 == 0
    assert r1 > 50, r1
    # aggregate within 20 % of 4 x one GPU's rate
    assert r4 >= 0.8 * 4 * r1, (r1, r4)
    if arch == "triton":
        # every model-server rank reports its CPU share and host plan (affinity.rank_info_metrics)
        assert len(texts) == 4
        for g, t in enumerate(texts):
            assert f'arena_rank_usable_cpus{{arch="triton",gpu="{g}"' in t
            assert f'arena_rank_threads{{arch="triton",gpu="{g}",role="decode_threads"}}' in t
