"""Monolithic HTTP service: /predict schema, /health, errors, metrics (CPU, fake + CPU backends)."""
from __future__ import annotations

import numpy as np
import pytest
from fastapi.testclient import TestClient

from inference_arena_amd.data.synthetic import encode_jpeg, synthetic_images
from inference_arena_amd.engine.pipeline import ImageResult
from inference_arena_amd.server.backends import Backend, Overloaded
from inference_arena_amd.server.monolithic import create_app
from inference_arena_amd.server.multipart import encode_multipart, parse_multipart
from inference_arena_amd.utils.settings import Settings


class FakeBackend(Backend):
    def __init__(self, fail=None):
        self.fail = fail
        self.calls = 0

    async def infer(self, image):
        self.calls += 1
        if self.fail:
            raise self.fail
        h, w = image.shape[:2]
        k = 2
        return ImageResult(boxes=np.array([[1, 2, 30, 40], [5, 5, w, h]], np.float32),
                           scores=np.array([0.9, 0.6], np.float32), classes=np.array([3, 7], np.int32),
                           topk_idx=np.array([[5, 1, 2, 3, 4], [999, 0, 1, 2, 3]], np.int32),
                           topk_logit=np.full((k, 5), 2.5, np.float32), topk_prob=np.full((k, 5), 0.25, np.float32),
                           det_count=k), {"detection_ms": 1.0, "classification_ms": 0.5, "batch_size": 1.0}


def _client(backend, **kw):
    s = Settings(LOG_LEVEL="WARNING", **kw)
    return TestClient(create_app(s, backend))


def test_multipart_roundtrip():
    body, ctype = encode_multipart("file", b"\x00\x01payload\r\n--x", "a.jpg")
    parts = parse_multipart(body, ctype)
    assert parts["file"] == (b"\x00\x01payload\r\n--x", "a.jpg")


def test_predict_schema_and_health():
    img = synthetic_images(1, 3)[0]
    body, ctype = encode_multipart("file", encode_jpeg(img))
    with _client(FakeBackend()) as c:
        assert c.get("/health").json() == {"status": "healthy", "models_loaded": True}
        r = c.post("/predict", content=body, headers={"content-type": ctype})
        assert r.status_code == 200, r.text
        js = r.json()
        assert set(js) == {"request_id", "detections", "timing"}
        assert {"detection_ms", "classification_ms", "total_ms"} <= set(js["timing"])
        d0 = js["detections"][0]
        assert set(d0["detection"]) == {"x1", "y1", "x2", "y2", "confidence", "class_id"}
        assert d0["classification"] == {"class_id": 5, "class_name": "electric ray", "confidence": 2.5}
        assert js["detections"][1]["classification"]["class_name"] == "toilet tissue"
        m = c.get("/metrics").text
        assert 'arena_requests_total{arch="monolithic",status="ok"} 1.0' in m


def test_predict_errors():
    with _client(FakeBackend()) as c:
        r = c.post("/predict", content=b"garbage", headers={"content-type": "image/jpeg"})
        assert r.status_code == 500 and "Failed to decode" in r.json()["detail"]
        body, ctype = encode_multipart("other", b"x")
        assert c.post("/predict", content=body, headers={"content-type": ctype}).status_code == 422
    img = encode_jpeg(synthetic_images(1, 4)[0])
    with _client(FakeBackend(fail=Overloaded("queue full"))) as c:
        body, ctype = encode_multipart("file", img)
        assert c.post("/predict", content=body, headers={"content-type": ctype}).status_code == 503


def test_fault_injection():
    img = encode_jpeg(synthetic_images(1, 4)[0])
    body, ctype = encode_multipart("file", img)
    with _client(FakeBackend(), ARENA_FAULT_EVERY=2) as c:
        codes = [c.post("/predict", content=body, headers={"content-type": ctype}).status_code for _ in range(4)]
    assert codes == [200, 500, 200, 500]


@pytest.mark.slow
def test_cpu_reference_backend_end_to_end(models):
    from inference_arena_amd.server.backends import CpuReferenceBackend

    be = CpuReferenceBackend(*models, threads=2)
    img = synthetic_images(1, 21)[0]
    body, ctype = encode_multipart("file", encode_jpeg(img, 95))
    with _client(be) as c:
        r = c.post("/predict", content=body, headers={"content-type": ctype})
        assert r.status_code == 200, r.text
        assert r.json()["timing"]["total_ms"] > 0


def test_device_fault_marks_instance_unhealthy():
    """A HIP error from the native batcher takes the instance out of rotation: /health -> 503
    (the replica router drops it), while ordinary request errors do not."""
    from inference_arena_amd.server.batching import AsyncBatcher, is_device_fault

    class FakeNativeBatcher:
        def __init__(self):
            self.errors = []

        def enqueue(self, x, cb):
            cb({"error": self.errors.pop(0) if self.errors else "", "det": np.zeros((0, 6), np.float32)})
            return 1

    ab = AsyncBatcher.__new__(AsyncBatcher)
    ab._b, ab._closed, ab.device_error = FakeNativeBatcher(), False, None
    ab._b.errors = ["submit: batch exceeds the staging pool",
                    "HIP error an illegal memory access was encountered at executor.cpp:700"]
    with pytest.raises(RuntimeError, match="staging pool"):
        ab.run_sync(np.zeros((2, 2, 3), np.uint8))
    assert ab.healthy
    with pytest.raises(RuntimeError, match="HIP error"):
        ab.run_sync(np.zeros((2, 2, 3), np.uint8))
    assert not ab.healthy and is_device_fault(ab.device_error)

    class FaultedBackend(FakeBackend):
        device_error = "HIP error hipErrorLaunchFailure"

        def ready(self):
            return False

    with _client(FaultedBackend()) as c:
        r = c.get("/health")
        assert r.status_code == 503 and r.json() == {"status": "unhealthy", "models_loaded": False}
    with _client(FakeBackend()) as c:
        assert c.get("/health").json() == {"status": "healthy", "models_loaded": True}
