"""Arm B device crop hand-off (``ARENA_CROP_TRANSPORT=device``).

The reference encodes every crop as JPEG q95 on the detection side and ships it through gRPC
(architectures/microservices/detection/app/grpc_client.py:99-168); the classification service decodes it
again (classification/app/servicer.py:65-76).  Here the decoded frame goes once into a ring of device
memory the detection process shares by IPC (csrc/runtime/ipc_buffer.h, hipIpcGetMemHandle over dmabuf); the
``ClassifyBatch`` RPC carries the ring's 64-byte handle, the frame's offset and size and the boxes
(``DeviceImageRef`` + ``source_box``); the classification service maps the ring once per detection process,
batches the frames of concurrent requests (from every detection process) and runs crop gather + MobileNetV2 on
them straight from the mapped memory (``Executor.submit_device``: device-to-device copies into its staging,
peer copies across GPUs).  JPEG stays the reference-compatible default; the protocol fields are additive.

Pieces:
  DeviceImageRing   detection side: slots of one IpcBuffer, ``put(image)`` -> (slot, DeviceImageRef)
  group_by_image    classification side: the crops of a batch request -> [(ref, boxes, crop indices)]
  DeviceClassifier  classification side: handle cache + micro-batcher over the split-classifier program
"""
from __future__ import annotations

import asyncio
import threading
import time
from dataclasses import dataclass

import numpy as np

from ..proto import inference_api as pb


@dataclass(frozen=True)
class ImageKey:
    handle: bytes
    device: int
    offset: int
    height: int
    width: int


class DeviceImageRing:
    """Fixed-size slots of one IPC-exported device buffer on the detection GPU.  ``put`` copies a decoded
    frame into a free slot (host -> device, synchronous, so the RPC that names it can go out right away);
    the slot is reused after ``release`` (the caller releases once the classification answer arrived)."""

    def __init__(self, slots: int, slot_bytes: int, device: int = 0, buffer=None):
        if buffer is None:
            from ..ops import native

            buffer = native().IpcBuffer(slots * slot_bytes, device)
        self.buf = buffer
        self.slots = slots
        self.slot_bytes = slot_bytes
        self.device = device
        self.handle = bytes(buffer.handle())
        self._free = list(range(slots - 1, -1, -1))
        self._cv = threading.Condition()

    def acquire(self, timeout: float = 30.0) -> int:
        with self._cv:
            if not self._cv.wait_for(lambda: self._free, timeout):
                raise TimeoutError("device image ring: no free slot")
            return self._free.pop()

    def try_acquire(self) -> int | None:
        with self._cv:
            return self._free.pop() if self._free else None

    def release(self, slot: int) -> None:
        with self._cv:
            self._free.append(slot)
            self._cv.notify()

    def slot_ptr(self, slot: int) -> int:
        """Device address of a slot (the detector exports its staged frame there: server/detection_service.py)."""
        return int(self.buf.ptr) + slot * self.slot_bytes

    def ref(self, slot: int, height: int, width: int) -> "pb.DeviceImageRef":
        if height * width * 3 > self.slot_bytes:
            raise ValueError(f"frame of {height * width * 3} bytes exceeds the ring slot ({self.slot_bytes})")
        return pb.DeviceImageRef(handle=self.handle, device=self.device, offset=slot * self.slot_bytes,
                                 height=height, width=width)

    def put(self, image: np.ndarray) -> tuple[int, "pb.DeviceImageRef"]:
        img = np.ascontiguousarray(image, dtype=np.uint8)
        if img.ndim != 3 or img.shape[2] != 3:
            raise ValueError(f"image must be HxWx3 uint8, got {img.shape}")
        if img.nbytes > self.slot_bytes:
            raise ValueError(f"image of {img.nbytes} bytes exceeds the ring slot ({self.slot_bytes})")
        slot = self.acquire()
        try:
            self.buf.write(slot * self.slot_bytes, img)
        except Exception:
            self.release(slot)
            raise
        ref = pb.DeviceImageRef(handle=self.handle, device=self.device, offset=slot * self.slot_bytes,
                                height=img.shape[0], width=img.shape[1])
        return slot, ref


def device_batch_request(request_id: str, ref, boxes: list[dict]):
    """One ``ClassifyBatch`` request for the crops of one frame: every crop names the frame and its box."""
    reqs = []
    for i, b in enumerate(boxes):
        r = pb.ClassificationRequest(request_id=f"{request_id}_{i}")
        r.device_image.CopyFrom(ref)
        r.source_box.x1, r.source_box.y1 = float(b["x1"]), float(b["y1"])
        r.source_box.x2, r.source_box.y2 = float(b["x2"]), float(b["y2"])
        r.source_box.confidence = float(b.get("confidence", 0.0))
        r.source_box.class_id = int(b.get("class_id", 0))
        reqs.append(r)
    return pb.BatchClassificationRequest(requests=reqs)


def group_by_image(requests) -> list[tuple[ImageKey, np.ndarray, list[int]]]:
    """Crops of a batch request that name device frames, grouped per frame (in first-seen order):
    (frame key, float32 [k, 6] boxes, indices of those crops in the request)."""
    groups: dict[ImageKey, tuple[list, list]] = {}
    for i, r in enumerate(requests):
        d = r.device_image
        key = ImageKey(bytes(d.handle), int(d.device), int(d.offset), int(d.height), int(d.width))
        b = r.source_box
        boxes, idx = groups.setdefault(key, ([], []))
        boxes.append((b.x1, b.y1, b.x2, b.y2, b.confidence, float(b.class_id)))
        idx.append(i)
    return [(k, np.asarray(bx, dtype=np.float32).reshape(-1, 6), ix) for k, (bx, ix) in groups.items()]


def is_device_request(r) -> bool:
    return r.HasField("device_image") and len(r.device_image.handle) > 0


class DeviceClassifier:
    """Classification side of the device transport: frames named by (IPC handle, offset) are mapped once per
    handle and classified in batches (up to ``max_batch`` frames and ``max_crops`` crops, ``max_delay_us`` to
    fill a batch; up to ``inflight`` batches on the device at once) by ``backend``, an object with
    ``submit(images, boxes) -> slot`` and ``collect(slot) -> dict`` (``engine.pipeline.GpuFrameClassifier``;
    tests pass a fake).  ``classify(key, boxes)`` resolves to per-crop (top-5 class ids, top-5 probabilities)."""

    def __init__(self, backend, open_handle, *, max_batch: int = 32, max_crops: int = 1 << 30,
                 max_delay_us: int = 300, inflight: int = 2, peer_check=None):
        self.backend = backend
        # peer_check(src_device): raises when this process's GPU cannot read a ring exported on src_device
        # (native require_peer_access: hipDeviceCanAccessPeer), so a cross-GPU reference gets a clear per-crop
        # error instead of a fault in the copy kernel
        self.peer_check = peer_check
        self._peer_ok: set[int] = set()
        # handle bytes -> device pointer, or (pointer, mapped bytes) (native ipc_open_range)
        self.open_handle = open_handle
        self.max_batch = max_batch
        self.max_crops = max_crops
        self.max_delay = max_delay_us * 1e-6
        self.inflight = inflight
        self._ptrs: dict[bytes, int] = {}
        self._queue: asyncio.Queue | None = None
        self._sem: asyncio.Semaphore | None = None
        self._task = None
        self._pool = None
        self.batches = 0
        self.frames = 0

    def _map(self, handle: bytes) -> tuple[int, int | None]:
        """(device address, mapped bytes or None when the opener does not report a size)."""
        m = self._ptrs.get(handle)
        if m is None:
            r = self.open_handle(handle)
            m = self._ptrs[handle] = (int(r[0]), int(r[1])) if isinstance(r, tuple) else (int(r), None)
        return m

    def _ptr(self, handle: bytes) -> int:
        return self._map(handle)[0]

    def validate(self, key: ImageKey, boxes: np.ndarray) -> None:
        """A frame reference must lie inside the exported ring and its boxes must be finite and in a sane range:
        the device copy and the crop plan trust both (a bad or stale DeviceImageRef would otherwise read out of
        bounds on the GPU and take down every in-flight batch).  Raises ValueError -> in-band per-crop error."""
        if key.height <= 0 or key.width <= 0 or key.offset < 0:
            raise ValueError(f"device frame: bad geometry {key.height}x{key.width} at offset {key.offset}")
        if self.peer_check is not None and key.device >= 0 and key.device not in self._peer_ok:
            try:
                self.peer_check(int(key.device))
            except RuntimeError as e:
                raise ValueError(f"device frame: {e}") from e
            self._peer_ok.add(int(key.device))
        _, size = self._map(key.handle)
        nbytes = key.height * key.width * 3
        if size is not None and key.offset + nbytes > size:
            raise ValueError(f"device frame: {nbytes} bytes at offset {key.offset} exceed the {size}-byte ring")
        b = np.asarray(boxes, dtype=np.float64)
        if b.ndim != 2 or b.shape[1] < 4 or not np.isfinite(b[:, :4]).all() or (np.abs(b[:, :4]) > 1e6).any():
            raise ValueError("device frame: box coordinates are not finite or out of range")

    async def classify(self, key: ImageKey, boxes: np.ndarray):
        self.validate(key, boxes)
        if self._queue is None:
            from concurrent.futures import ThreadPoolExecutor

            self._queue = asyncio.Queue()
            self._sem = asyncio.Semaphore(self.inflight)
            self._pool = ThreadPoolExecutor(max_workers=self.inflight, thread_name_prefix="frame-cls")
            self._task = asyncio.get_running_loop().create_task(self._run())
        fut = asyncio.get_running_loop().create_future()
        await self._queue.put((key, boxes, fut))
        return await fut

    async def _run(self):
        pending = None
        while True:
            first = pending if pending is not None else await self._queue.get()
            pending = None
            items, crops = [first], len(first[1])
            deadline = time.perf_counter() + self.max_delay
            while len(items) < self.max_batch:
                try:
                    nxt = self._queue.get_nowait()
                except asyncio.QueueEmpty:
                    left = deadline - time.perf_counter()
                    if left <= 0:
                        break
                    try:
                        nxt = await asyncio.wait_for(self._queue.get(), left)
                    except asyncio.TimeoutError:
                        break
                if crops + len(nxt[1]) > self.max_crops:
                    pending = nxt  # opens the next batch
                    break
                items.append(nxt)
                crops += len(nxt[1])
            # a waiter whose RPC was cancelled (deadline, client gone) no longer owns its frame: the detection side
            # may already have reused the ring slot, so its crops are dropped before they reach the device
            items = [it for it in items if not it[2].done()]
            if not items:
                continue
            await self._sem.acquire()
            asyncio.get_running_loop().create_task(self._dispatch(items))

    async def _dispatch(self, items):
        try:
            images = [(self._ptr(k.handle) + k.offset, k.height, k.width, k.device) for k, _, _ in items]
            boxes = [b for _, b, _ in items]
            res = await asyncio.get_running_loop().run_in_executor(self._pool, self._submit_collect, images, boxes)
            self.batches += 1
            self.frames += len(items)
            offs = res["crop_offset"]
            for i, (_, _, fut) in enumerate(items):
                a, b = int(offs[i]), int(offs[i + 1])
                if not fut.done():
                    fut.set_result(list(zip(res["topk_idx"][a:b].tolist(), res["topk_prob"][a:b].tolist())))
        except Exception as e:  # noqa: BLE001 — every waiter hears the failure
            for _, _, fut in items:
                if not fut.done():
                    fut.set_exception(e)
        finally:
            self._sem.release()

    def _submit_collect(self, images, boxes):
        return self.backend.collect(self.backend.submit(images, boxes))

    def close(self) -> None:
        if self._task is not None:
            self._task.cancel()
        if self._pool is not None:
            self._pool.shutdown(wait=False)
