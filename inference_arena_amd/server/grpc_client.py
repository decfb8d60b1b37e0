"""Async client of ``inference.ClassificationService`` (arm B detection side).

Reference: architectures/microservices/detection/app/grpc_client.py:52-168 —
``grpc.aio`` channel with 50 MB limits, ``connect`` waits for the channel to
be ready (30 s), ``classify`` encodes the crop (PIL JPEG q95) into a
``ClassificationRequest{request_id=f"{rid}_{i}", image_crop, source_box}``,
``classify_parallel`` fans all crops of a request out with
``asyncio.gather`` (the H1b mechanism).

Additions: ``transport`` selects jpeg (reference) / png / raw crops,
``classify_batch`` sends all crops in one ``ClassifyBatch`` RPC and
``classify_device`` sends one ``ClassifyBatch`` that names a device-resident
frame instead of carrying crops (``transport="device"``,
server/device_transport.py; crops of frames that do not fit the ring still
go as JPEG).
"""
from __future__ import annotations

import asyncio

import grpc
import numpy as np

from ..proto import inference_api as pb
from .classification_service import GRPC_OPTIONS
from .crop_codec import encode_crop
from .device_transport import device_batch_request


class ClassificationClient:
    def __init__(self, endpoint: str, transport: str = "jpeg", timeout_s: float = 30.0):
        self.endpoint = endpoint
        self.transport = transport
        self.codec = "jpeg" if transport == "device" else transport  # bytes fallback of the device transport
        self.timeout_s = timeout_s
        self.channel = None
        self.stub = None
        self.health = None

    async def connect(self, ready_timeout: float = 30.0) -> None:
        self.channel = grpc.aio.insecure_channel(self.endpoint, options=GRPC_OPTIONS)
        await asyncio.wait_for(self.channel.channel_ready(), timeout=ready_timeout)
        self.stub = pb.ClassificationService.stub(self.channel)
        self.health = pb.Health.stub(self.channel)

    async def close(self) -> None:
        if self.channel is not None:
            await self.channel.close()
            self.channel = None

    @property
    def connected(self) -> bool:
        return self.stub is not None

    def _request(self, rid: str, crop: np.ndarray, box: dict | None):
        req = pb.ClassificationRequest(request_id=rid, image_crop=encode_crop(crop, self.codec))
        if box:
            req.source_box.x1 = float(box["x1"])
            req.source_box.y1 = float(box["y1"])
            req.source_box.x2 = float(box["x2"])
            req.source_box.y2 = float(box["y2"])
            req.source_box.confidence = float(box["confidence"])
            req.source_box.class_id = int(box["class_id"])
        return req

    async def classify(self, rid: str, crop: np.ndarray, box: dict | None = None):
        try:
            return await self.stub.Classify(self._request(rid, crop, box), timeout=self.timeout_s)
        except grpc.aio.AioRpcError as e:
            return pb.ClassificationResponse(request_id=rid, error=f"{e.code().name}: {e.details()}")

    async def classify_parallel(self, request_id: str, crops: list[np.ndarray], boxes: list[dict]):
        return await asyncio.gather(*(self.classify(f"{request_id}_{i}", c, b)
                                      for i, (c, b) in enumerate(zip(crops, boxes))))

    async def classify_batch(self, request_id: str, crops: list[np.ndarray], boxes: list[dict]):
        return await self._batch(pb.BatchClassificationRequest(
            requests=[self._request(f"{request_id}_{i}", c, b) for i, (c, b) in enumerate(zip(crops, boxes))]))

    async def classify_device(self, request_id: str, ref, boxes: list[dict]):
        """All crops of one frame: ``ref`` (pb.DeviceImageRef) names the frame, ``boxes`` the crops."""
        return await self._batch(device_batch_request(request_id, ref, boxes))

    async def _batch(self, breq):
        try:
            return list((await self.stub.ClassifyBatch(breq, timeout=self.timeout_s)).responses)
        except grpc.aio.AioRpcError as e:
            return [pb.ClassificationResponse(request_id=r.request_id, error=f"{e.code().name}: {e.details()}")
                    for r in breq.requests]

    async def check_health(self) -> bool:
        r = await self.health.Check(pb.HealthCheckRequest(), timeout=self.timeout_s)
        return r.status == pb.SERVING


class ClassificationClientPool:
    """Detection-side view of several classification services (one per GPU: scripts/start_arena.py
    ``--arch microservices --gpus N``).  ``CLASSIFICATION_GRPC_ENDPOINT`` may list endpoints separated by
    commas; each crop RPC goes to the endpoint with the fewest outstanding RPCs (ties: round robin), so the
    fan-out of one request spreads over the classification GPUs.  Same interface as
    ``ClassificationClient``."""

    def __init__(self, endpoints: list[str], transport: str = "jpeg", timeout_s: float = 30.0):
        if not endpoints:
            raise ValueError("no classification endpoints")
        self.clients = [ClassificationClient(e, transport, timeout_s) for e in endpoints]
        self.endpoint = ",".join(endpoints)
        self.transport = transport
        self.outstanding = [0] * len(self.clients)
        self._rr = 0

    async def connect(self, ready_timeout: float = 30.0) -> None:
        await asyncio.gather(*(c.connect(ready_timeout) for c in self.clients))

    async def close(self) -> None:
        await asyncio.gather(*(c.close() for c in self.clients))

    @property
    def connected(self) -> bool:
        return all(c.connected for c in self.clients)

    def pick(self) -> int:
        n = len(self.clients)
        best = min(range(n), key=lambda k: (self.outstanding[(self._rr + k) % n], k))
        i = (self._rr + best) % n
        self._rr = (i + 1) % n
        return i

    async def _on(self, i: int, coro):
        self.outstanding[i] += 1
        try:
            return await coro
        finally:
            self.outstanding[i] -= 1

    async def classify(self, rid: str, crop: np.ndarray, box: dict | None = None):
        i = self.pick()
        return await self._on(i, self.clients[i].classify(rid, crop, box))

    async def classify_parallel(self, request_id: str, crops: list[np.ndarray], boxes: list[dict]):
        return await asyncio.gather(*(self.classify(f"{request_id}_{i}", c, b)
                                      for i, (c, b) in enumerate(zip(crops, boxes))))

    async def classify_batch(self, request_id: str, crops: list[np.ndarray], boxes: list[dict]):
        i = self.pick()
        return await self._on(i, self.clients[i].classify_batch(request_id, crops, boxes))

    async def classify_device(self, request_id: str, ref, boxes: list[dict]):
        i = self.pick()
        return await self._on(i, self.clients[i].classify_device(request_id, ref, boxes))

    async def check_health(self) -> bool:
        return all(await asyncio.gather(*(c.check_health() for c in self.clients)))


def make_classification_client(spec: str, transport: str = "jpeg", timeout_s: float = 30.0):
    """One client for a single endpoint, a least-outstanding pool for a comma-separated list."""
    eps = [e.strip() for e in spec.split(",") if e.strip()]
    if len(eps) == 1:
        return ClassificationClient(eps[0], transport, timeout_s)
    return ClassificationClientPool(eps, transport, timeout_s)
