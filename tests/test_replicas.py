"""Multi-process data-parallel serving on CPU: 2 replicas (gloo group for the
start-up broadcast) sharing one SO_REUSEPORT port; and the RCCL/gloo blob
broadcast helper at world size 2."""
from __future__ import annotations

import json
import os
import subprocess
import sys
import urllib.request

import pytest

from inference_arena_amd.data.synthetic import encode_jpeg, synthetic_images
from inference_arena_amd.parallel.replicas import free_port, launch
from inference_arena_amd.server.multipart import encode_multipart

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_broadcast_blob_world2():
    code = r"""
import numpy as np, torch.distributed as dist
from inference_arena_amd.parallel import dist as D
info = D.init_from_env("gloo")
blob = np.arange(1000, dtype=np.uint8) if info.rank == 0 else None
out = D.broadcast_blob(blob, info)
assert out.nbytes == 1000 and out[999] == 999 % 256
obj = D.broadcast_object({"a": 1} if info.rank == 0 else None, info)
assert obj == {"a": 1}
assert D.allreduce_max(float(info.rank), info) == 1.0
g = D.allgather_floats([float(info.rank)] * 2, info)
assert g == [[0.0, 0.0], [1.0, 1.0]]
D.barrier(info); D.shutdown(info)
print("ok", info.rank)
"""
    port = free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), PYTHONPATH=ROOT)
        procs.append(subprocess.Popen([sys.executable, "-c", code], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    outs = [p.communicate(timeout=120)[0] for p in procs]
    assert all(p.returncode == 0 for p in procs), outs
    assert "ok 0" in outs[0] and "ok 1" in outs[1]


@pytest.mark.slow
def test_two_cpu_replicas_share_port(tmp_path):
    port = free_port()
    rep = launch("monolithic", 2, port=port, env={"ARENA_DEVICE": "cpu", "LOG_LEVEL": "WARNING",
                                                   "PYTHONPATH": ROOT}, log_dir=str(tmp_path))
    try:
        assert rep.wait_ready(240), [open(tmp_path / f"replica_{r}.log").read()[-2000:] for r in range(2)]
        body, ctype = encode_multipart("file", encode_jpeg(synthetic_images(1, 3, hw=(96, 128))[0]))
        seen = set()
        for _ in range(40):  # fresh connection per request -> kernel spreads them over replicas
            req = urllib.request.Request(f"http://127.0.0.1:{port}/predict", data=body,
                                         headers={"content-type": ctype})
            with urllib.request.urlopen(req, timeout=60) as r:
                assert r.status == 200
                seen.add(r.headers["x-arena-replica"])
                assert "detections" in json.loads(r.read())
            if len(seen) == 2:
                break
        assert seen == {"0", "1"}
    finally:
        rep.stop()


def test_router_least_outstanding():
    import asyncio

    from inference_arena_amd.server.router import Router

    r = Router(["a:1", "b:2", "c:3"])
    r.inflight.update({"http://a:1": 3, "http://b:2": 1, "http://c:3": 1})
    picks = {r.pick() for _ in range(4)}
    assert picks == {"http://b:2", "http://c:3"}
    r.healthy["http://b:2"] = False
    assert r.pick() == "http://c:3"
    asyncio.run(asyncio.sleep(0))


def test_router_forwards_to_live_replicas(tmp_path):
    """Router over two fake monolithic services on separate ports."""
    from fastapi.testclient import TestClient

    from tests.test_loadgen import _serve
    from tests.test_server_monolithic import FakeBackend

    from inference_arena_amd.server.monolithic import create_app as mono
    from inference_arena_amd.server.router import create_app
    from inference_arena_amd.utils.settings import Settings

    servers = [_serve(mono(Settings(LOG_LEVEL="WARNING"), FakeBackend())) for _ in range(2)]
    try:
        app = create_app([f"127.0.0.1:{p}" for _, _, p in servers])
        body, ctype = encode_multipart("file", encode_jpeg(synthetic_images(1, 3, hw=(64, 64))[0]))
        with TestClient(app) as c:
            for _ in range(6):
                r = c.post("/predict", content=body, headers={"content-type": ctype})
                assert r.status_code == 200 and len(r.json()["detections"]) == 2
            served = c.get("/router/stats").json()["served"]
        assert sum(served.values()) == 6 and all(v >= 1 for v in served.values())
    finally:
        for s, t, _ in servers:
            s.should_exit = True
            t.join(10)


def test_supervise_keeps_rank_and_backs_off(tmp_path):
    """A restarted replica keeps its port / tag (ARENA_REPLICA_RANK = its original rank), the first restart is
    immediate, further ones back off exponentially, and a crash-looping replica is left down after
    max_restarts (restarts came back as rank 0 every 0.5 s forever)."""
    import time

    from inference_arena_amd.parallel.replicas import Replicas

    # each "replica" writes its ARENA_REPLICA_RANK and exits 3 (a device fault) at once
    out = tmp_path / "ranks.txt"
    argv = [sys.executable, "-c",
            f"import os; open({str(out)!r}, 'a').write(os.environ['ARENA_REPLICA_RANK'] + '\\n'); raise SystemExit(3)"]
    procs = [subprocess.Popen([sys.executable, "-c", "raise SystemExit(3)"]) for _ in range(2)]
    for p in procs:
        p.wait()
    specs = [(argv, {"RANK": str(r), "PATH": os.environ.get("PATH", "")}, r, None) for r in range(2)]
    rep = Replicas(procs, 8100, 1, specs, max_restarts=3, backoff_s=1.0, healthy_s=60.0)  # > a loaded spawn
    assert rep.supervise() == 2  # first restart: immediate
    for p in rep.procs:
        p.wait()
    assert rep.supervise() == 0  # inside the backoff window
    deadline = time.time() + 30
    while len(rep.given_up) < 2 and time.time() < deadline:
        rep.supervise()
        for p in rep.procs:
            p.wait()
        time.sleep(0.05)
    assert rep.given_up == {0, 1} and rep.restarts == 6  # 3 restarts each, then left down
    assert sorted(out.read_text().split()) == ["0", "0", "0", "1", "1", "1"]
