"""asyncio / thread front of the native DynamicBatcher (csrc/runtime/batcher.cpp).

``AsyncBatcher`` owns a DynamicBatcher over the executors of one or more
``GpuProgramRunner`` instances (the Triton ``instance_group.count``
equivalent).  ``await run(x)`` enqueues one input (uint8 HxWx3 image or fp32
[3,S,S] tensor) and resolves when its batch has been collected; the C++
worker threads call back with the GIL only for the result conversion, so the
event loop never blocks on GPU work.  ``run_sync`` is the same for threads
(sync gRPC handlers).
"""
from __future__ import annotations

import asyncio
import threading

import numpy as np


class Overloaded(RuntimeError):
    """The request queue is full (HTTP 503 / gRPC RESOURCE_EXHAUSTED)."""


class TooLarge(ValueError):
    """The input exceeds what one batch can stage on the device (HTTP 413 / gRPC INVALID_ARGUMENT)."""


def _enqueue_or_raise(rid: int) -> None:
    if rid == -2:
        raise TooLarge("input larger than the device staging pool of one batch")
    if rid < 0:
        raise Overloaded("inference queue full")


def is_device_fault(message: str) -> bool:
    """A HIP runtime error (ARENA_HIP_CHECK in csrc/kernels/common.h): the device context of this
    process is no longer trustworthy, so the instance must be taken out of service (SURVEY.md §5
    failure detection: "a HIP error marks the instance unhealthy")."""
    return message.startswith("HIP error")


class AsyncBatcher:
    def __init__(self, runners, *, max_batch: int, preferred: list[int] | None = None,
                 max_queue_delay_us: int = 500, max_queue_size: int = 4096, idle_queue_delay_us: int = -1,
                 overlap: int = -1):
        from ..ops import native

        self.runners = list(runners)
        self.max_batch = int(max_batch)
        self._b = native().DynamicBatcher([r.ex for r in self.runners], {
            "max_batch": self.max_batch,
            "preferred": sorted(int(p) for p in (preferred or []) if int(p) <= self.max_batch),
            "max_queue_delay_us": int(max_queue_delay_us),
            "max_queue_size": int(max_queue_size),
            "idle_queue_delay_us": int(idle_queue_delay_us),  # -1: max_queue_delay_us (batcher.h)
            "overlap": int(overlap),  # -1: ARENA_BATCH_OVERLAP (default 0); batcher.h BatcherConfig.overlap
        })
        self._closed = False
        self.device_error: str | None = None  # first HIP error seen; the instance is unhealthy from then on

    def _check(self, d: dict) -> dict:
        err = d["error"]
        if err:
            if self.device_error is None and is_device_fault(err):
                self.device_error = err
            raise RuntimeError(err)
        return d

    @property
    def healthy(self) -> bool:
        return self.device_error is None

    @staticmethod
    def _prep(x: np.ndarray) -> np.ndarray:
        if x.dtype == np.uint8:
            return np.ascontiguousarray(x)
        return np.ascontiguousarray(x, dtype=np.float32)

    async def run(self, x: np.ndarray, export_to: int = 0) -> dict:
        """``export_to``: device address on the instance's GPU that receives the staged frame (D2D, in the
        batch's stream order) — complete when this returns."""
        loop = asyncio.get_running_loop()
        fut: asyncio.Future = loop.create_future()

        def done(d):
            loop.call_soon_threadsafe(lambda: fut.done() or fut.set_result(d))

        _enqueue_or_raise(self._b.enqueue(self._prep(x), done, int(export_to)))
        return self._check(await fut)

    async def run_jpeg(self, data: bytes, decode, threads: int = 4, export_to: int = 0) -> dict:
        """An encoded upload through the native split decoder (csrc/runtime/jpeg_ingest.h: Huffman decode on C++
        threads into pinned memory, frame reconstructed on the GPU inside the batch); formats it does not cover
        go through ``await decode(data)`` (the caller's PIL path) and ``run``.  Decode failures raise
        ValueError / TooLarge like the PIL path."""
        if getattr(self, "_ingest", None) is None:
            from ..ops import native
            from ..processing.transforms import max_image_pixels

            self._ingest = native().JpegIngest(self._b, {"threads": int(threads),
                                                         "max_image_pixels": int(max_image_pixels())})
        loop = asyncio.get_running_loop()
        fut: asyncio.Future = loop.create_future()

        def done(d):
            loop.call_soon_threadsafe(lambda: fut.done() or fut.set_result(("ok", d)))

        def fallback():
            loop.call_soon_threadsafe(lambda: fut.done() or fut.set_result(("fallback", None)))

        self._ingest.submit(data, done, fallback, int(export_to))
        kind, d = await fut
        if kind == "fallback":
            return await self.run(await decode(data), export_to=export_to)
        err = d["error"]
        if err.startswith("Failed to decode image"):
            raise (TooLarge(err) if "image too large" in err else ValueError(err))
        if err == "request queue is full":
            raise Overloaded(err)
        if err.startswith("image exceeds"):
            raise TooLarge(err)
        return self._check(d)

    def ingest_stats(self) -> dict | None:
        ing = getattr(self, "_ingest", None)
        return dict(ing.stats()) if ing is not None else None

    async def run_many(self, xs: list[np.ndarray]) -> list[dict]:
        return list(await asyncio.gather(*(self.run(x) for x in xs)))

    def run_sync(self, x: np.ndarray, timeout: float | None = 60.0) -> dict:
        ev = threading.Event()
        box: list = []

        def done(d):
            box.append(d)
            ev.set()

        _enqueue_or_raise(self._b.enqueue(self._prep(x), done))
        if not ev.wait(timeout):
            raise TimeoutError("inference timed out")
        return self._check(box[0])

    def stats(self) -> dict:
        return dict(self._b.stats())

    def close(self) -> None:
        if not self._closed:
            self._closed = True
            if getattr(self, "_ingest", None) is not None:
                self._ingest.stop()
            self._b.shutdown()
