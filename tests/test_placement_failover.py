"""Multi-GPU placement of every arm (Triton instance_group semantics, per-GPU classification
services, split topology plan), the detection side's classification channel pool, and replica
failover (device fault -> replica exits -> supervisor starts a fresh process).  CPU only."""
from __future__ import annotations

import asyncio

import numpy as np
import os
import sys
import time
import urllib.error
import urllib.request

import pytest

from inference_arena_amd.parallel.placement import endpoints, instance_devices, parse_gpu_list

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))


def test_parse_gpu_list():
    assert parse_gpu_list("0,2,1") == [0, 1, 2]
    assert parse_gpu_list("0-3") == [0, 1, 2, 3]
    assert parse_gpu_list("1-2,5") == [1, 2, 5]
    assert parse_gpu_list("", default=3) == [3]
    assert parse_gpu_list(None) == [0]
    assert parse_gpu_list([4, 4, 1]) == [1, 4]
    assert endpoints("a:1, b:2,,") == ["a:1", "b:2"]


def test_instance_group_semantics():
    # count instances on EACH listed GPU (Triton); no list = every visible GPU; KIND_CPU -> default device
    assert instance_devices([{"count": 2, "kind": "KIND_GPU", "gpus": [0, 1]}], n_visible=8) == [0, 0, 1, 1]
    assert instance_devices([{"count": 1, "kind": "KIND_GPU", "gpus": []}], n_visible=4) == [0, 1, 2, 3]
    assert instance_devices([{"count": 1, "kind": "KIND_CPU"}], default_gpu=2, n_visible=4) == [2]
    assert instance_devices([{"count": 1, "kind": "KIND_GPU", "gpus": [3]},
                             {"count": 2, "kind": "KIND_GPU", "gpus": [5]}], n_visible=8) == [3, 5, 5]
    assert instance_devices([], default_gpu=1, n_visible=2) == [1]
    with pytest.raises(ValueError, match="only 2 visible"):
        instance_devices([{"count": 1, "kind": "KIND_GPU", "gpus": [4]}], n_visible=2)


def test_instance_group_from_generated_config():
    from inference_arena_amd.repository import model_config as mc

    cfg = mc.parse(mc.dump(mc.generate("yolov5n", gpus=[0, 1, 2, 3])))
    assert list(cfg.instance_group[0].gpus) == [0, 1, 2, 3]
    assert instance_devices(list(cfg.instance_group), n_visible=4) == [0, 1, 2, 3]
    ref = mc.parse(mc.dump(mc.generate("yolov5n", reference_compat=True, gpus=[0, 1])))
    assert list(ref.instance_group[0].gpus) == []  # the reference's config carries no device list


def test_microservices_gpu_plan():
    from start_arena import plan_microservices

    p = plan_microservices(4)
    assert p["detection_gpus"] == [0, 1, 2, 3]
    assert p["classification"] == [(0, 8201), (1, 8211), (2, 8221), (3, 8231)]
    assert p["endpoint"].split(",") == ["127.0.0.1:8201", "127.0.0.1:8211", "127.0.0.1:8221", "127.0.0.1:8231"]
    s = plan_microservices(8, split=True)
    assert s["detection_gpus"] == [0, 1, 2, 3] and [g for g, _ in s["classification"]] == [4, 5, 6, 7]
    assert plan_microservices(1, split=True)["detection_gpus"] == [0]
    from start_arena import _queue_env, hw_queues_per_process

    # hardware queues per process when several GPU processes share a device (HIP default 4 up to 3 processes)
    assert [hw_queues_per_process(n) for n in (1, 3, 4, 5, 6, 11)] == [None, None, 2, 2, 1, 1]
    assert _queue_env({}, 5) == {"GPU_MAX_HW_QUEUES": "2"} and _queue_env({}, 2) == {}
    assert _queue_env({"GPU_MAX_HW_QUEUES": "4"}, 5) == {"GPU_MAX_HW_QUEUES": "2"}  # inherited default: capped
    assert _queue_env({"ARENA_HW_QUEUES": "3"}, 5)["GPU_MAX_HW_QUEUES"] == "3"  # explicit arena override wins
    m = plan_microservices(2, cls_procs_per_gpu=3)  # several classification processes per GPU
    assert m["classification"] == [(0, 8201), (0, 8202), (0, 8203), (1, 8211), (1, 8212), (1, 8213)]
    assert len(m["endpoint"].split(",")) == 6


def test_classification_pool_least_outstanding():
    from inference_arena_amd.server.grpc_client import (ClassificationClient, ClassificationClientPool,
                                                        make_classification_client)

    assert isinstance(make_classification_client("127.0.0.1:1"), ClassificationClient)
    pool = make_classification_client("127.0.0.1:1,127.0.0.1:2,127.0.0.1:3")
    assert isinstance(pool, ClassificationClientPool) and len(pool.clients) == 3
    pool.outstanding = [2, 0, 1]
    assert pool.pick() == 1
    pool.outstanding = [0, 0, 0]
    picks = [pool.pick() for _ in range(6)]
    assert sorted(picks) == [0, 0, 1, 1, 2, 2]  # ties rotate

    class Fake:
        def __init__(self, k):
            self.k, self.calls = k, 0

        async def classify(self, rid, crop, box=None):
            self.calls += 1
            await asyncio.sleep(0.01)
            return self.k

    pool.clients = [Fake(k) for k in range(3)]
    out = asyncio.run(pool.classify_parallel("r", [None] * 9, [None] * 9))
    assert sorted(out) == [0, 0, 0, 1, 1, 1, 2, 2, 2]  # one request's fan-out spread over every service
    assert pool.outstanding == [0, 0, 0]


def _get(url, data=None, headers=None, timeout=60):
    req = urllib.request.Request(url, data=data, headers=headers or {})
    try:
        with urllib.request.urlopen(req, timeout=timeout) as r:
            return r.status
    except urllib.error.HTTPError as e:
        return e.code


@pytest.mark.slow
def test_replica_restarts_after_device_fault(tmp_path):
    """A device fault takes the replica out (503, socket closed, exit 3); the supervisor starts a fresh
    process on the same GPU and port, which serves again."""
    from inference_arena_amd.data.synthetic import encode_jpeg, synthetic_images
    from inference_arena_amd.parallel.replicas import free_port, launch
    from inference_arena_amd.server.multipart import encode_multipart

    port = free_port()
    rep = launch("monolithic", 1, port=port, log_dir=str(tmp_path),
                 env={"ARENA_DEVICE": "cpu", "LOG_LEVEL": "WARNING", "PYTHONPATH": ROOT, "ARENA_FAULT_EVERY": "2",
                      "ARENA_FAULT_MODE": "device"})
    try:
        assert rep.wait_ready(240), open(tmp_path / "replica_0.log").read()[-3000:]
        pid0 = rep.procs[0].pid
        body, ctype = encode_multipart("file", encode_jpeg(synthetic_images(1, 3, hw=(64, 96))[0]))
        url = f"http://127.0.0.1:{port}/predict"
        codes = [_get(url, body, {"content-type": ctype}) for _ in range(2)]
        assert codes == [200, 500], codes
        t0 = time.time()
        while rep.procs[0].poll() is None and time.time() - t0 < 30:
            time.sleep(0.2)
        assert rep.procs[0].returncode == 3, open(tmp_path / "replica_0.log").read()[-3000:]
        assert rep.supervise() == 1 and rep.restarts == 1
        assert rep.procs[0].pid != pid0
        assert rep.wait_ready(240), open(tmp_path / "replica_0.log").read()[-3000:]
        assert _get(url, body, {"content-type": ctype}) == 200  # the fresh process serves
    finally:
        rep.stop()


def test_async_decode_pool_processes():
    """The servers' DecodePool with spawned decode processes (ARENA_DECODE_PROCS) decodes like the
    thread path, and reports undecodable uploads."""
    from inference_arena_amd.data.synthetic import encode_jpeg, synthetic_images
    from inference_arena_amd.processing.transforms import load_image_from_bytes
    from inference_arena_amd.server.app_common import DecodePool

    jpegs = [encode_jpeg(im) for im in synthetic_images(4, 9, hw=(48, 64))]

    async def go():
        pool = DecodePool(procs=2)
        try:
            out = await asyncio.gather(*(pool.decode(j) for j in jpegs))
            with pytest.raises(ValueError):
                await pool.decode(b"not an image")
            return out
        finally:
            pool.close()

    out = asyncio.run(go())
    for j, im in zip(jpegs, out):
        assert np.array_equal(im, load_image_from_bytes(j))
