"""Arm C on CPU: config.pbtxt schema, model repository, the KServe-v2 model
server (gRPC + HTTP + metrics, fp32 CPU device) and the gateway in both modes."""
from __future__ import annotations

import asyncio
import json
import socket
import threading

import numpy as np
import pytest
import torch
from fastapi.testclient import TestClient

from inference_arena_amd.data.synthetic import encode_jpeg, synthetic_images
from inference_arena_amd.labels import load_labels
from inference_arena_amd.proto import kserve as kv
from inference_arena_amd.repository import model_config as mc
from inference_arena_amd.repository import store

REFERENCE_STYLE = """
# reference-style config (template of infrastructure/minio/triton_config.py)
name: "yolov5n"
platform: "onnxruntime_onnx"
max_batch_size: 0
input [{
  name: "images"
  data_type: TYPE_FP32
  dims: [ 1, 3, 640, 640 ]
}]
output [{ name: "output0"  data_type: TYPE_FP32  dims: [ 1, 84, 8400 ] }]
instance_group [{ count: 1  kind: KIND_CPU }]
parameters [
  { key: "intra_op_thread_count"  value: { string_value: "2" } },
  { key: "inter_op_thread_count"  value: { string_value: "1" } }
]
"""


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_config_roundtrip_and_reference_syntax():
    cfg = mc.parse(REFERENCE_STYLE)
    assert list(cfg.input[0].dims) == [1, 3, 640, 640] and cfg.max_batch_size == 0
    assert cfg.instance_group[0].kind == mc.Kind.Value("KIND_CPU")
    assert cfg.parameters["intra_op_thread_count"].string_value == "2"
    assert mc.validate(cfg) == []
    for name in ("yolov5n", "mobilenetv2"):
        for compat in (False, True):
            c = mc.generate(name, reference_compat=compat)
            assert mc.validate(c) == []
            assert mc.parse(mc.dump(c)) == c
    c = mc.generate("yolov5n")
    assert c.max_batch_size == 32 and list(c.input[0].dims) == [3, 640, 640]
    assert list(c.dynamic_batching.preferred_batch_size) == [8, 16, 32]
    assert list(mc.generate("yolov5n", reference_compat=True).input[0].dims) == [1, 3, 640, 640]
    assert mc.validate(mc.generate_pipeline()) == []


def test_config_errors():
    with pytest.raises(mc.ConfigError):
        mc.parse('name: "x"\nbogus_field: 3\n')
    bad = mc.parse('name: "x"\nplatform: "arena_hip"\nmax_batch_size: 0\ndynamic_batching { }\n'
                   'input [{ name: "a" data_type: TYPE_FP32 dims: [0] }]')
    errs = mc.validate(bad)
    assert any("output" in e for e in errs) and any("instance_group" in e for e in errs)
    assert any("dynamic_batching" in e for e in errs) and any("invalid dims" in e for e in errs)


@pytest.fixture(scope="module")
def repo(tmp_path_factory):
    root = tmp_path_factory.mktemp("model_repository")
    store.build_repository(root, seed=0)
    return root


def test_repository_layout_verify_sync(repo, tmp_path):
    assert (repo / "yolov5n" / "1" / "model.safetensors").exists()
    meta = json.loads((repo / "mobilenetv2" / "metadata.json").read_text())
    assert meta["sha256"] == store.sha256_file(repo / "mobilenetv2" / "1" / "model.safetensors")
    assert meta["input"]["shape"] == [1, 3, 224, 224]
    assert all(v == [] for v in store.verify_repository(repo).values())
    assert "checksums.txt" in {p.name for p in repo.iterdir()}
    # second build keeps files (idempotent, reference "skip if exists")
    assert set(store.build_repository(repo, seed=0)["yolov5n"]) == {"present"}
    dst = tmp_path / "copy"
    copied = store.sync_repository(repo, dst)
    assert "yolov5n/config.pbtxt" in copied and store.sync_repository(repo, dst) == []
    assert (dst / "arena_pipeline" / "1").is_dir()
    # corrupt the copy -> sha256 mismatch is reported
    f = dst / "yolov5n" / "1" / "model.safetensors"
    f.write_bytes(f.read_bytes()[:-1] + b"\x00")
    assert store.verify_repository(dst)["yolov5n"] == ["sha256 mismatch"]
    flat = store.init_flat(repo, tmp_path / "flat")
    assert sorted(p.name for p in flat) == ["mobilenetv2.safetensors", "yolov5n.safetensors"]
    # weights load into the same networks the zoo builds
    from inference_arena_amd.models.zoo import default_models

    m = store.load_module(repo / "mobilenetv2" / "1" / "model.safetensors")
    x = torch.randn(1, 3, 224, 224)
    with torch.no_grad():
        assert torch.allclose(m(x), default_models(0)[1].eval()(x), atol=1e-5)


class ServerThread:
    def __init__(self, repo):
        from inference_arena_amd.server.model_server import start_grpc
        from inference_arena_amd.server.modelserver_core import ModelServer

        self.ms = ModelServer(repo, device="cpu")
        self.port = _free_port()
        self.loop = asyncio.new_event_loop()
        ready = threading.Event()

        async def boot():
            self.g, _ = await start_grpc(self.ms, "127.0.0.1", self.port)
            ready.set()

        self.t = threading.Thread(target=lambda: (self.loop.run_until_complete(boot()), self.loop.run_forever()),
                                  daemon=True)
        self.t.start()
        assert ready.wait(30)

    def stop(self):
        asyncio.run_coroutine_threadsafe(self.g.stop(0), self.loop).result(10)
        self.loop.call_soon_threadsafe(self.loop.stop)
        self.t.join(10)
        self.ms.close()


@pytest.fixture(scope="module")
def model_server(repo):
    s = ServerThread(repo)
    yield s
    s.stop()


def test_grpc_kserve_protocol(model_server):
    from inference_arena_amd.server.kserve_client import ModelServerClient

    x1 = np.random.default_rng(0).standard_normal((1, 3, 224, 224)).astype(np.float32)
    x2 = np.random.default_rng(1).standard_normal((2, 3, 224, 224)).astype(np.float32)

    async def go():
        import grpc

        c = ModelServerClient(f"127.0.0.1:{model_server.port}")
        assert await c.wait_for_server_ready(10)
        live = (await c.stub.ServerLive(kv.ServerLiveRequest())).live
        md = await c.get_model_metadata("yolov5n")
        idx = await c.stub.RepositoryIndex(kv.RepositoryIndexRequest())
        y1 = await c.infer_mobilenet(x1)
        y2 = (await c.infer("mobilenetv2", {"input": x2}))["output"]
        errs = []
        for call in (c.infer("nope", {"input": x1}), c.infer("mobilenetv2", {"input": x1[:, :, :100]}),
                     c.infer("mobilenetv2", {"input": x1.astype(np.float64)})):
            try:
                await call
            except grpc.aio.AioRpcError as e:
                errs.append(e.code().name)
        st = await c.stub.ModelStatistics(kv.ModelStatisticsRequest(name="mobilenetv2"))
        await c.close()
        return live, md, idx, y1, y2, errs, st

    live, md, idx, y1, y2, errs, st = asyncio.run(go())
    assert live
    assert md["inputs"][0]["name"] == "images" and md["inputs"][0]["shape"] == [-1, 3, 640, 640]
    assert md["outputs"][0]["shape"] == [-1, 84, 8400]
    assert {m.name for m in idx.models} == {"yolov5n", "mobilenetv2", "arena_pipeline"}
    ref = model_server.ms.models["mobilenetv2"].module
    with torch.no_grad():
        np.testing.assert_allclose(y1, ref(torch.from_numpy(x1)).numpy(), rtol=1e-4, atol=1e-4)
        np.testing.assert_allclose(y2, ref(torch.from_numpy(x2)).numpy(), rtol=1e-4, atol=1e-4)
    assert y2.shape == (2, 1000)
    assert errs == ["NOT_FOUND", "INVALID_ARGUMENT", "INVALID_ARGUMENT"]
    assert st.model_stats[0].inference_count == 3 and st.model_stats[0].execution_count == 2


def test_http_kserve_and_metrics(model_server):
    from inference_arena_amd.server.model_server import create_http_app, create_metrics_app

    app = create_http_app(model_server.ms)
    x = np.random.default_rng(2).standard_normal((1, 3, 224, 224)).astype(np.float32)
    with TestClient(app) as c:
        assert c.get("/v2/health/ready").status_code == 200
        assert c.get("/v2/models/mobilenetv2").json()["platform"] == "arena_hip"
        assert c.get("/v2/models/nope").status_code == 404
        js = c.post("/v2/models/mobilenetv2/infer", json={
            "id": "a", "inputs": [{"name": "input", "shape": [1, 3, 224, 224], "datatype": "FP32",
                                   "data": x.ravel().tolist()}]}).json()
        y_json = np.asarray(js["outputs"][0]["data"], np.float32).reshape(js["outputs"][0]["shape"])
        # binary tensor extension, both directions
        header = json.dumps({"inputs": [{"name": "input", "shape": [1, 3, 224, 224], "datatype": "FP32",
                                         "parameters": {"binary_data_size": x.nbytes}}],
                             "outputs": [{"name": "output", "parameters": {"binary_data": True}}]}).encode()
        r = c.post("/v2/models/mobilenetv2/infer", content=header + x.tobytes(),
                   headers={"Inference-Header-Content-Length": str(len(header))})
        n = int(r.headers["inference-header-content-length"])
        y_bin = np.frombuffer(r.content[n:], np.float32).reshape(1, 1000)
        bad = c.post("/v2/models/mobilenetv2/infer", json={"inputs": [{"name": "input", "shape": [2],
                                                                       "datatype": "FP32", "data": [1.0]}]})
        assert bad.status_code == 400
        stats = c.get("/v2/models/mobilenetv2/stats").json()
    assert js["id"] == "a" and js["model_name"] == "mobilenetv2"
    np.testing.assert_allclose(y_json, y_bin, rtol=1e-6)
    assert stats["model_stats"][0]["inference_count"] >= 2
    with TestClient(create_metrics_app(model_server.ms)) as c:
        text = c.get("/metrics").text
    assert 'nv_inference_count_total{model="mobilenetv2",version="1"}' in text


def _gateway_predict(model_server, mode):
    from inference_arena_amd.server.gateway import create_app
    from inference_arena_amd.server.multipart import encode_multipart
    from inference_arena_amd.utils.settings import Settings

    s = Settings(LOG_LEVEL="WARNING", TRITON_GRPC_ENDPOINT=f"127.0.0.1:{model_server.port}",
                 ARENA_GATEWAY_MODE=mode, TRITON_TIMEOUT_SECONDS=30)
    from inference_arena_amd.data.curator import workload_images

    img = workload_images(1)[0]
    body, ctype = encode_multipart("file", encode_jpeg(img))
    with TestClient(create_app(s)) as c:
        assert c.get("/health").json()["models_loaded"] is True
        r = c.post("/predict", content=body, headers={"content-type": ctype})
        assert r.status_code == 200, r.text
        js = r.json()
    assert {"detection_ms", "classification_ms", "total_ms"} <= set(js["timing"])
    for d in js["detections"]:
        assert set(d["detection"]) == {"x1", "y1", "x2", "y2", "confidence", "class_id"}
        assert d["classification"]["class_name"] in set(load_labels())
    return js


def test_gateway_modes_agree(model_server):
    """The fused ensemble and the reference per-model protocol give the same detections (CPU fp32)."""
    a = _gateway_predict(model_server, "pipeline")
    b = _gateway_predict(model_server, "tensor")
    assert len(a["detections"]) >= 3
    da = [(round(d["detection"]["x1"], 1), d["classification"]["class_id"]) for d in a["detections"]]
    db = [(round(d["detection"]["x1"], 1), d["classification"]["class_id"]) for d in b["detections"]]
    assert sorted(da) == sorted(db)


def test_gateway_native_handler_front_matches_fastapi(model_server):
    """ARENA_NATIVE_HTTP=1 gateway (server/native_handler.py): the C++ HTTP layer + the same predict_bytes
    coroutine give the FastAPI route's detections; /health answers natively."""
    import asyncio
    import http.client
    import json
    import threading

    from inference_arena_amd.data.curator import workload_images
    from inference_arena_amd.server.gateway import create_app
    from inference_arena_amd.server.multipart import encode_multipart
    from inference_arena_amd.server.native_handler import serve_app
    from inference_arena_amd.utils.settings import Settings

    ref = _gateway_predict(model_server, "pipeline")
    s = Settings(LOG_LEVEL="WARNING", TRITON_GRPC_ENDPOINT=f"127.0.0.1:{model_server.port}",
                 ARENA_GATEWAY_MODE="pipeline", TRITON_TIMEOUT_SECONDS=30)
    box, ready = {}, threading.Event()
    loop = asyncio.new_event_loop()

    async def main():
        box["stop"] = asyncio.Event()
        box["rc"] = await serve_app(create_app(s), port=0, host="127.0.0.1", stop=box["stop"],
                                    on_ready=lambda srv: (box.__setitem__("srv", srv), ready.set()))

    t = threading.Thread(target=lambda: loop.run_until_complete(main()), daemon=True)
    t.start()
    assert ready.wait(60)
    try:
        body, ctype = encode_multipart("file", encode_jpeg(workload_images(1)[0]))
        c = http.client.HTTPConnection("127.0.0.1", box["srv"].port, timeout=60)
        c.request("POST", "/predict", body=body, headers={"Content-Type": ctype})
        r = c.getresponse()
        js = json.loads(r.read())
        assert r.status == 200, js
        c.request("GET", "/health")
        h = c.getresponse()
        assert h.status == 200 and json.loads(h.read())["status"] == "healthy"
        c.close()
    finally:
        loop.call_soon_threadsafe(box["stop"].set)
        t.join(30)
    assert box["rc"] == 0
    got = sorted((round(d["detection"]["x1"], 1), d["classification"]["class_id"]) for d in js["detections"])
    want = sorted((round(d["detection"]["x1"], 1), d["classification"]["class_id"]) for d in ref["detections"])
    assert got == want and len(got) >= 3


def test_model_server_process_stops_cleanly_on_signals(repo):
    """SIGINT / SIGTERM: the model server stops accepting, drains (5 s grace), closes its backends and exits 0 —
    no KeyboardInterrupt traceback and no shared-memory segment left behind (VERDICT round 2, weak item 9;
    reference: architectures/microservices/classification/app/main.py:86-104)."""
    import os
    import signal
    import subprocess
    import sys
    import time
    import urllib.request
    from pathlib import Path

    root = Path(__file__).resolve().parents[1]
    for sig in (signal.SIGINT, signal.SIGTERM):
        shm_before = set(os.listdir("/dev/shm"))
        ports = [_free_port() for _ in range(3)]
        env = dict(os.environ, ARENA_DEVICE="cpu", PYTHONPATH=str(root), LOG_LEVEL="WARNING", ARENA_DECODE_PROCS="2")
        p = subprocess.Popen([sys.executable, "-m", "inference_arena_amd.server.model_server", "--model-repository",
                              str(repo), "--device", "cpu", "--http-port", str(ports[0]), "--grpc-port",
                              str(ports[1]), "--metrics-port", str(ports[2])],
                             env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
        try:
            t0 = time.time()
            while time.time() - t0 < 180:
                try:
                    with urllib.request.urlopen(f"http://127.0.0.1:{ports[0]}/v2/health/ready", timeout=2) as r:
                        if r.status == 200:
                            break
                except OSError:
                    time.sleep(0.3)
            # the segments this server (and its decode workers) map, not whatever other tests create meanwhile
            owned = set()
            for pid in [p.pid] + _children(p.pid):
                try:
                    for line in open(f"/proc/{pid}/maps"):
                        if "/dev/shm/" in line:
                            owned.add(line.split("/dev/shm/")[1].split()[0])
                except OSError:
                    pass
            p.send_signal(sig)
            out, _ = p.communicate(timeout=60)
        finally:
            if p.poll() is None:
                p.kill()
        assert p.returncode == 0, out[-2000:]
        assert "Traceback" not in out, out[-2000:]
        assert owned, "the server maps no shared memory (decode pool missing?)"
        assert not (owned & (set(os.listdir("/dev/shm")) - shm_before)), "shared memory leaked"


def _children(pid: int) -> list[int]:
    import os

    out = []
    for d in os.listdir("/proc"):
        if d.isdigit():
            try:
                with open(f"/proc/{d}/stat") as f:
                    if int(f.read().rsplit(")", 1)[1].split()[1]) == pid:
                        out.append(int(d))
            except (OSError, ValueError, IndexError):
                pass
    return out
