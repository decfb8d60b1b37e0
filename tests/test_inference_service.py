"""``inference.InferenceService/Infer`` (declared, never implemented upstream:
src/shared/proto/inference.proto:137-152) over a live grpc.aio server with a
fake pipeline backend (CPU)."""
from __future__ import annotations

import asyncio
import socket
import threading

import grpc
import numpy as np
import pytest

from inference_arena_amd.data.synthetic import encode_jpeg, synthetic_images
from inference_arena_amd.engine.pipeline import ImageResult
from inference_arena_amd.proto import inference_api as pb
from inference_arena_amd.server.backends import Backend
from inference_arena_amd.server.inference_service import select_detections
from inference_arena_amd.utils.settings import Settings


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class FakePipeline(Backend):
    """Three detections (class-asc / score-desc order) with distinct top-5s."""

    def __init__(self):
        self.shapes = []

    async def infer(self, image):
        self.shapes.append(image.shape)
        boxes = np.array([[0, 0, 10, 10], [1, 1, 20, 20], [2, 2, 30, 30]], np.float32)
        scores = np.array([0.9, 0.6, 0.8], np.float32)
        classes = np.array([0, 0, 3], np.int32)
        idx = np.array([[7, 1, 2, 3, 4], [8, 1, 2, 3, 4], [9, 1, 2, 3, 4]], np.int32)
        logit = np.tile(np.array([5, 4, 3, 2, 1], np.float32), (3, 1))
        prob = np.tile(np.array([0.5, 0.2, 0.1, 0.1, 0.1], np.float32), (3, 1))
        return ImageResult(boxes, scores, classes, idx, logit, prob, det_count=3), {}


class Server:
    def __init__(self, backend, via_classification: bool):
        self.port = _free_port()
        self.loop = asyncio.new_event_loop()
        ready = threading.Event()
        s = Settings(LOG_LEVEL="WARNING", HOST="127.0.0.1")

        async def boot():
            if via_classification:
                from inference_arena_amd.server.classification_service import start_server

                from test_microservices import FakeClassifier

                self.server, self.servicer, _ = await start_server(s, FakeClassifier(), port=self.port,
                                                                   pipeline_backend=backend)
            else:
                from inference_arena_amd.server.inference_service import start_server

                self.server, self.servicer, _ = await start_server(s, backend, port=self.port)
            ready.set()

        self.t = threading.Thread(target=lambda: (self.loop.run_until_complete(boot()), self.loop.run_forever()),
                                  daemon=True)
        self.t.start()
        assert ready.wait(20)

    def stop(self):
        asyncio.run_coroutine_threadsafe(self.server.stop(0), self.loop).result(10)
        self.loop.call_soon_threadsafe(self.loop.stop)
        self.t.join(10)


def _infer(port: int, req):
    with grpc.insecure_channel(f"127.0.0.1:{port}") as ch:
        return pb.InferenceService.stub(ch).Infer(req, timeout=20)


@pytest.mark.parametrize("via_classification", [False, True])
def test_infer_returns_detections_with_classifications(via_classification):
    be = FakePipeline()
    srv = Server(be, via_classification)
    try:
        img = synthetic_images(1, 5)[0]
        resp = _infer(srv.port, pb.InferenceRequest(request_id="r1", image=encode_jpeg(img, quality=95)))
        assert resp.error == ""
        assert resp.request_id == "r1"
        assert [r.detection.class_id for r in resp.results] == [0, 0, 3]
        assert [r.classification.class_id for r in resp.results] == [7, 8, 9]
        assert resp.results[0].classification.confidence == pytest.approx(0.5)  # softmax convention
        assert resp.results[2].detection.x2 == pytest.approx(30.0)
        assert resp.timing.total_ms >= resp.timing.inference_ms >= 0
        assert be.shapes == [img.shape]
    finally:
        srv.stop()


def test_infer_threshold_and_max_detections():
    srv = Server(FakePipeline(), False)
    try:
        img = encode_jpeg(synthetic_images(1, 6)[0], quality=95)
        r = _infer(srv.port, pb.InferenceRequest(request_id="a", image=img, detection_threshold=0.7))
        assert [round(x.detection.confidence, 2) for x in r.results] == [0.9, 0.8]
        r = _infer(srv.port, pb.InferenceRequest(request_id="b", image=img, max_detections=1))
        assert len(r.results) == 1 and r.results[0].detection.confidence == pytest.approx(0.9)
    finally:
        srv.stop()


def test_infer_reports_errors_in_band():
    srv = Server(FakePipeline(), False)
    try:
        r = _infer(srv.port, pb.InferenceRequest(request_id="bad", image=b"not an image"))
        assert r.request_id == "bad" and r.error != "" and len(r.results) == 0
        r = _infer(srv.port, pb.InferenceRequest(request_id="empty"))
        assert "empty" in r.error
    finally:
        srv.stop()


def test_health_check_on_inference_server():
    srv = Server(FakePipeline(), False)
    try:
        with grpc.insecure_channel(f"127.0.0.1:{srv.port}") as ch:
            st = pb.Health.stub(ch).Check(pb.HealthCheckRequest(service="inference"), timeout=10)
        assert st.status == pb.SERVING
    finally:
        srv.stop()


def test_select_detections_keeps_pipeline_order():
    s = np.array([0.9, 0.55, 0.8, 0.7], np.float32)
    assert select_detections(s, 0.0, 0).tolist() == [0, 1, 2, 3]
    assert select_detections(s, 0.6, 0).tolist() == [0, 2, 3]
    assert select_detections(s, 0.0, 2).tolist() == [0, 2]
    assert select_detections(s, 0.75, 5).tolist() == [0, 2]
