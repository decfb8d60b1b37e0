"""Arm B (microservices) on CPU: proto contract, crop transport, the gRPC
classification service (fake + CPU-reference backends) and the detection
service's /predict fan-out over a live gRPC server."""
from __future__ import annotations

import asyncio
import socket
import threading

import numpy as np
import pytest
from fastapi.testclient import TestClient

from inference_arena_amd.data.synthetic import encode_jpeg, synthetic_images
from inference_arena_amd.proto import inference_api as pb
from inference_arena_amd.server.crop_codec import decode_crop, encode_crop
from inference_arena_amd.server.multipart import encode_multipart
from inference_arena_amd.server.service_backends import ClassifierBackend, DetectorBackend
from inference_arena_amd.utils.settings import Settings


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class FakeClassifier(ClassifierBackend):
    def __init__(self):
        self.shapes = []

    async def classify(self, crop):
        self.shapes.append(crop.shape)
        cid = int(crop.shape[0] % 1000)
        return (np.array([cid, 1, 2, 3, 4], np.int32), np.array([5, 4, 3, 2, 1], np.float32),
                np.array([0.6, 0.2, 0.1, 0.05, 0.05], np.float32))


class FakeDetector(DetectorBackend):
    async def detect(self, image):
        h, w = image.shape[:2]
        return np.array([[0, 0, 10, 20, 0.9, 1], [5, 5, w, h, 0.7, 2], [3, 3, 3, 9, 0.6, 4]], np.float32), {}


class ServerThread:
    """Classification gRPC server running on its own event loop thread."""

    def __init__(self, backend, **settings):
        from inference_arena_amd.server.classification_service import start_server

        self.port = _free_port()
        self.loop = asyncio.new_event_loop()
        self.ready = threading.Event()
        s = Settings(LOG_LEVEL="WARNING", HOST="127.0.0.1", **settings)

        async def boot():
            self.server, self.servicer, _ = await start_server(s, backend, port=self.port)
            self.ready.set()

        self.t = threading.Thread(target=lambda: (self.loop.run_until_complete(boot()), self.loop.run_forever()),
                                  daemon=True)
        self.t.start()
        assert self.ready.wait(20)

    def stop(self):
        asyncio.run_coroutine_threadsafe(self.server.stop(0), self.loop).result(10)
        self.loop.call_soon_threadsafe(self.loop.stop)
        self.t.join(10)


@pytest.fixture()
def fake_server():
    srv = ServerThread(FakeClassifier())
    yield srv
    srv.stop()


def test_proto_field_numbers_match_reference_contract():
    """Field numbers / types of the reference inference.proto:30-152 (wire compatibility)."""
    def fields(msg):
        return {f.name: f.number for f in msg.DESCRIPTOR.fields}

    assert fields(pb.BoundingBox) == {"x1": 1, "y1": 2, "x2": 3, "y2": 4, "confidence": 5, "class_id": 6}
    # + the arena's device-frame extension (field 100; reference peers skip it as an unknown field)
    assert fields(pb.ClassificationRequest) == {"request_id": 1, "image_crop": 2, "source_box": 3, "device_image": 100}
    assert fields(pb.ClassificationResponse) == {"request_id": 1, "result": 2, "top_k": 3, "timing": 4, "error": 5}
    assert fields(pb.TimingInfo) == {"preprocessing_ms": 1, "inference_ms": 2, "postprocessing_ms": 3, "total_ms": 4}
    assert fields(pb.InferenceRequest) == {"request_id": 1, "image": 2, "detection_threshold": 3,
                                           "max_detections": 4, "top_k": 5}
    assert pb.ClassificationService.path("ClassifyBatch") == "/inference.ClassificationService/ClassifyBatch"
    # hand-encoded bytes of ClassificationRequest{request_id:"r", image_crop:b"\x01"}
    assert pb.ClassificationRequest(request_id="r", image_crop=b"\x01").SerializeToString() == b"\n\x01r\x12\x01\x01"


@pytest.mark.parametrize("transport", ["raw", "png", "jpeg"])
def test_crop_codec(transport):
    crop = synthetic_images(1, 9)[0][:37, :53]
    back = decode_crop(encode_crop(crop, transport))
    assert back.shape == crop.shape and back.dtype == np.uint8
    if transport == "jpeg":
        assert np.abs(back.astype(int) - crop.astype(int)).mean() < 8
    else:
        assert np.array_equal(back, crop)


def test_crop_codec_gray_and_rgba():
    import io

    from PIL import Image

    g = np.arange(64, dtype=np.uint8).reshape(8, 8)
    buf = io.BytesIO()
    Image.fromarray(g).save(buf, format="PNG")
    assert decode_crop(buf.getvalue()).shape == (8, 8, 3)
    buf = io.BytesIO()
    Image.fromarray(np.zeros((4, 5, 4), np.uint8), "RGBA").save(buf, format="PNG")
    assert decode_crop(buf.getvalue()).shape == (4, 5, 3)
    with pytest.raises(ValueError):
        decode_crop(b"ARW1" + b"\x00" * 3)


def test_classify_rpcs_and_health(fake_server):
    from inference_arena_amd.server.grpc_client import ClassificationClient

    async def go():
        cl = ClassificationClient(f"127.0.0.1:{fake_server.port}", transport="raw")
        await cl.connect(10)
        crops = [np.full((h, 7, 3), 9, np.uint8) for h in (11, 12, 13)]
        boxes = [{"x1": 0, "y1": 0, "x2": 7, "y2": h, "confidence": 0.9, "class_id": 1} for h in (11, 12, 13)]
        par = await cl.classify_parallel("rq", crops, boxes)
        bat = await cl.classify_batch("rq", crops, boxes)
        bad = await cl.classify("bad", np.zeros((2, 2, 3), np.uint8))
        cl.transport = "jpeg"
        healthy = await cl.check_health()
        # garbage bytes -> in-band error, not an RPC failure
        raw = await cl.stub.Classify(pb.ClassificationRequest(request_id="x", image_crop=b"not an image"))
        await cl.close()
        return par, bat, bad, healthy, raw

    par, bat, bad, healthy, raw = asyncio.run(go())
    assert [r.request_id for r in par] == ["rq_0", "rq_1", "rq_2"]
    assert [r.result.class_id for r in par] == [11, 12, 13] == [r.result.class_id for r in bat]
    assert par[0].result.class_name == "goldfinch"
    assert abs(par[0].result.confidence - 0.6) < 1e-6 and len(par[0].top_k) == 5
    assert par[0].timing.total_ms > 0
    assert bad.error == "" and healthy
    assert raw.error and raw.request_id == "x"


def test_classification_service_cpu_reference_backend():
    """The CPU fp32 backend returns softmax top-5 in descending order."""
    from inference_arena_amd.models.zoo import make_mobilenet
    from inference_arena_amd.server.service_backends import CpuClassifierBackend

    be = CpuClassifierBackend(make_mobilenet(1), threads=2)
    idx, logit, prob = asyncio.run(be.classify(synthetic_images(1, 2)[0][:100, :80]))
    be.close()
    assert idx.shape == (5,) and np.all(np.diff(logit) <= 0) and np.all(np.diff(prob) <= 0)
    assert 0 < prob[0] <= 1


@pytest.mark.parametrize("fanout", ["parallel", "batch"])
def test_detection_service_predict(fake_server, fanout):
    from inference_arena_amd.server.detection_service import create_app

    s = Settings(LOG_LEVEL="WARNING", CLASSIFICATION_GRPC_ENDPOINT=f"127.0.0.1:{fake_server.port}",
                 ARENA_FANOUT=fanout, ARENA_CROP_TRANSPORT="png")
    img = synthetic_images(1, 5)[0]
    body, ctype = encode_multipart("file", encode_jpeg(img))
    with TestClient(create_app(s, detector=FakeDetector())) as c:
        assert c.get("/health").json() == {"status": "healthy", "models_loaded": True}
        r = c.post("/predict", content=body, headers={"content-type": ctype})
        assert r.status_code == 200, r.text
        js = r.json()
    assert {"detection_ms", "classification_ms", "total_ms"} <= set(js["timing"])
    dets = js["detections"]
    assert len(dets) == 3
    # crop sizes travel intact: class id = crop height % 1000; zero-width box -> 1x1 black crop
    h, w = img.shape[:2]
    assert [d["classification"]["class_id"] for d in dets] == [20, h - 5, 1]
    assert dets[0]["classification"]["confidence"] == pytest.approx(0.6)
    assert dets[1]["detection"]["class_id"] == 2


def test_detection_service_drops_failed_crops():
    """A classification server that is down -> every crop errors in-band and is dropped (reference)."""
    from inference_arena_amd.server.detection_service import create_app
    from inference_arena_amd.server.grpc_client import ClassificationClient

    srv = ServerThread(FakeClassifier())
    port = srv.port
    s = Settings(LOG_LEVEL="WARNING", CLASSIFICATION_GRPC_ENDPOINT=f"127.0.0.1:{port}")
    body, ctype = encode_multipart("file", encode_jpeg(synthetic_images(1, 6)[0]))
    cl = ClassificationClient(f"127.0.0.1:{port}", timeout_s=2.0)
    with TestClient(create_app(s, detector=FakeDetector(), client=cl)) as c:
        assert c.post("/predict", content=body, headers={"content-type": ctype}).status_code == 200
        srv.stop()
        r = c.post("/predict", content=body, headers={"content-type": ctype})
        assert r.status_code == 200 and r.json()["detections"] == []


def _native_serve(app, port=0):
    """Run ``native_handler.serve_app`` on a thread; returns (server, stop, thread)."""
    from inference_arena_amd.server.native_handler import serve_app

    box, ready = {}, threading.Event()
    loop = asyncio.new_event_loop()

    async def main():
        box["stop"] = asyncio.Event()
        box["rc"] = await serve_app(app, port=port, host="127.0.0.1", stop=box["stop"],
                                    on_ready=lambda srv: (box.__setitem__("srv", srv), ready.set()))

    t = threading.Thread(target=lambda: loop.run_until_complete(main()), daemon=True)
    t.start()
    assert ready.wait(30)
    return box, loop, t


def test_detection_service_native_handler_front(fake_server):
    """ARENA_NATIVE_HTTP=1 detection service: C++ HTTP/multipart, Python handler (take/complete): same JSON
    as the FastAPI route, concurrent keep-alive clients, 422 / 404 / health / metrics."""
    import http.client
    import json
    import time

    from inference_arena_amd.server.detection_service import create_app

    s = Settings(LOG_LEVEL="WARNING", CLASSIFICATION_GRPC_ENDPOINT=f"127.0.0.1:{fake_server.port}",
                 ARENA_FANOUT="batch", ARENA_CROP_TRANSPORT="raw")
    img = synthetic_images(1, 5)[0]
    body, ctype = encode_multipart("file", encode_jpeg(img))
    box, loop, t = _native_serve(create_app(s, detector=FakeDetector()))
    port = box["srv"].port
    try:
        c = http.client.HTTPConnection("127.0.0.1", port, timeout=30)
        c.request("POST", "/predict", body=body, headers={"Content-Type": ctype})
        r = c.getresponse()
        js = json.loads(r.read())
        assert r.status == 200, js
        h, w = img.shape[:2]
        assert [d["classification"]["class_id"] for d in js["detections"]] == [20, h - 5, 1]
        assert {"detection_ms", "classification_ms", "total_ms"} <= set(js["timing"])
        # a raw JPEG body works too; an empty multipart field is a 422 from the native layer
        c.request("POST", "/predict", body=encode_jpeg(img), headers={"Content-Type": "image/jpeg"})
        r = c.getresponse()
        assert r.status == 200 and len(json.loads(r.read())["detections"]) == 3
        bad, bct = encode_multipart("other", b"x")
        c.request("POST", "/predict", body=bad, headers={"Content-Type": bct})
        r = c.getresponse()
        assert r.status == 422 and "detail" in json.loads(r.read())
        # undecodable upload -> the handler's 500 with {"detail": ...}
        c.request("POST", "/predict", body=b"not a jpeg", headers={"Content-Type": "image/jpeg"})
        r = c.getresponse()
        assert r.status == 500 and json.loads(r.read())["detail"]
        c.request("GET", "/nope")
        r = c.getresponse()
        r.read()
        assert r.status == 404
        errors, ok = [], []

        def worker():
            try:
                cc = http.client.HTTPConnection("127.0.0.1", port, timeout=30)
                for _ in range(8):
                    cc.request("POST", "/predict", body=body, headers={"Content-Type": ctype})
                    rr = cc.getresponse()
                    assert rr.status == 200 and len(json.loads(rr.read())["detections"]) == 3
                    ok.append(1)
                cc.close()
            except Exception as e:  # noqa: BLE001
                errors.append(e)

        ts = [threading.Thread(target=worker) for _ in range(6)]
        for th in ts:
            th.start()
        for th in ts:
            th.join()
        assert not errors and len(ok) == 48
        st = box["srv"].stats()
        assert st["ok"] >= 50 and st["detections"] >= 150 and st["bad_request"] >= 1 and st["errors"] >= 1
        deadline = time.monotonic() + 5
        while True:
            c.request("GET", "/metrics")
            r = c.getresponse()
            text = r.read().decode()
            if "arena_requests_total" in text or time.monotonic() > deadline:
                break
            time.sleep(0.3)
        assert r.status == 200 and "arena_requests_total" in text
        c.request("GET", "/health")
        r = c.getresponse()
        assert r.status == 200 and json.loads(r.read())["models_loaded"] is True
        c.close()
    finally:
        loop.call_soon_threadsafe(box["stop"].set)
        t.join(30)
    assert box["rc"] == 0


def test_native_handler_drains_in_flight_requests_on_stop():
    """Shutdown of the handler-mode front end: the listening socket goes first (new connections are refused),
    a request already inside the (slow) handler is still answered."""
    import http.client
    import json
    import time


    from fastapi import FastAPI

    from inference_arena_amd.server.schemas import PredictResponse

    app = FastAPI()
    entered = threading.Event()

    async def slow_predict(data: bytes):
        entered.set()
        await asyncio.sleep(0.6)
        return PredictResponse(request_id="r", detections=[], timing={"total_ms": 600.0})

    app.state.arena = {"predict_bytes": slow_predict, "healthy": lambda: True, "metrics": None}
    box, loop, t = _native_serve(app)
    port = box["srv"].port
    got = {}

    def client():
        c = http.client.HTTPConnection("127.0.0.1", port, timeout=30)
        c.request("POST", "/predict", body=b"x", headers={"Content-Type": "image/jpeg"})
        r = c.getresponse()
        got["status"], got["body"] = r.status, json.loads(r.read())

    th = threading.Thread(target=client)
    th.start()
    assert entered.wait(20)  # the request is inside slow_predict (not a fixed sleep: loaded CI machines)
    loop.call_soon_threadsafe(box["stop"].set)
    # drained: the port stops accepting (polled: a loaded host can take longer than a fixed sleep to get there)
    deadline, refused = time.monotonic() + 10.0, False
    while not refused and time.monotonic() < deadline:
        time.sleep(0.05)
        try:
            socket.create_connection(("127.0.0.1", port), timeout=2).close()
        except OSError:
            refused = True
    assert refused, "the listening socket still accepts after stop"
    th.join(10)
    t.join(30)
    assert got.get("status") == 200 and got["body"]["request_id"] == "r"
    assert box["rc"] == 0



def test_cancelled_detection_keeps_its_ring_slot_until_the_batch_lands():
    """a request cancelled while its native batch still holds export_dst = the ring slot must not hand
    the slot back before that batch has copied its frame; released from the detection's completion instead."""
    import asyncio

    from inference_arena_amd.server.detection_service import _detect_holding_slot

    class Ring:
        def __init__(self):
            self.released = []

        def release(self, s):
            self.released.append(s)

    async def main():
        ring = Ring()
        gate = asyncio.Event()

        async def detect():
            await gate.wait()  # the batch is queued / on the device
            return [], {}

        outer = asyncio.ensure_future(_detect_holding_slot(detect(), ring, 3))
        await asyncio.sleep(0.01)
        outer.cancel()
        try:
            await outer
        except asyncio.CancelledError:
            pass
        assert ring.released == []  # still owned by the in-flight batch
        gate.set()
        await asyncio.sleep(0.01)
        assert ring.released == [3]

        async def boom():
            raise RuntimeError("device fault")

        try:
            await _detect_holding_slot(boom(), ring, 5)
        except RuntimeError:
            pass
        assert ring.released == [3, 5]  # failed detection: released at once
        assert await _detect_holding_slot(detect(), ring, None) == ([], {})

    asyncio.run(main())
