"""Async KServe-v2 gRPC client of the model server (tritonclient replacement).

Reference: architectures/triton/gateway/app/triton_client.py:18-184 —
``wait_for_server_ready`` with exponential backoff capped at 10 s,
``infer_yolo`` / ``infer_mobilenet`` with hard-validated input shapes
``(1,3,640,640)`` / ``(1,3,224,224)``, ``get_model_metadata``.  tritonclient
is not installed; this client speaks the same protocol with the arena's
``proto.kserve`` messages over ``grpc.aio`` (so the gateway's event loop is
not blocked by a synchronous client as in the reference).
"""
from __future__ import annotations

import asyncio
import time

import grpc
import numpy as np

from ..proto import kserve as kv
from .model_server import GRPC_OPTIONS


class ModelServerClient:
    def __init__(self, endpoint: str, timeout_s: float = 60.0):
        self.endpoint = endpoint
        self.timeout_s = timeout_s
        self.channel = grpc.aio.insecure_channel(endpoint, options=GRPC_OPTIONS)
        self.stub = kv.GRPCInferenceService.stub(self.channel)

    async def close(self) -> None:
        await self.channel.close()

    async def is_server_ready(self) -> bool:
        try:
            return (await self.stub.ServerReady(kv.ServerReadyRequest(), timeout=5.0)).ready
        except grpc.aio.AioRpcError:
            return False

    async def wait_for_server_ready(self, timeout_s: float = 60.0) -> bool:
        t0, delay = time.monotonic(), 0.25
        while time.monotonic() - t0 < timeout_s:
            if await self.is_server_ready():
                return True
            await asyncio.sleep(delay)
            delay = min(delay * 2, 10.0)
        return False

    async def get_model_metadata(self, name: str) -> dict:
        r = await self.stub.ModelMetadata(kv.ModelMetadataRequest(name=name), timeout=self.timeout_s)
        tm = lambda t: {"name": t.name, "datatype": t.datatype, "shape": list(t.shape)}  # noqa: E731
        return {"name": r.name, "versions": list(r.versions), "platform": r.platform,
                "inputs": [tm(t) for t in r.inputs], "outputs": [tm(t) for t in r.outputs]}

    async def infer(self, model: str, inputs: dict[str, np.ndarray], outputs: list[str] | None = None,
                    request_id: str = "") -> dict[str, np.ndarray]:
        req = kv.make_infer_request(model, inputs, outputs, request_id)
        return kv.decode_outputs(await self.stub.ModelInfer(req, timeout=self.timeout_s))

    async def infer_yolo(self, tensor: np.ndarray, model: str = "yolov5n") -> np.ndarray:
        if tensor.shape != (1, 3, 640, 640):
            raise ValueError(f"YOLO input must be (1, 3, 640, 640), got {tensor.shape}")
        return (await self.infer(model, {"images": tensor.astype(np.float32)}, ["output0"]))["output0"]

    async def infer_mobilenet(self, tensor: np.ndarray, model: str = "mobilenetv2") -> np.ndarray:
        if tensor.shape != (1, 3, 224, 224):
            raise ValueError(f"MobileNet input must be (1, 3, 224, 224), got {tensor.shape}")
        return (await self.infer(model, {"input": tensor.astype(np.float32)}, ["output"]))["output"]

    async def infer_pipeline(self, image_bytes: bytes, model: str = "arena_pipeline",
                             request_id: str = "") -> dict[str, np.ndarray]:
        a = np.empty(1, dtype=object)
        a[0] = image_bytes
        return await self.infer(model, {"IMAGE_BYTES": a}, None, request_id)
