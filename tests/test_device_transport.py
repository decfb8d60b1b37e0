"""Arm B device crop hand-off (server/device_transport.py) on CPU: the handle protocol, the frame ring, the
classification side's per-frame grouping and micro-batching, and /predict end to end over a live gRPC server —
with a fake device (a host bytearray per IPC handle) standing in for hipIpc* and the frame classifier."""
from __future__ import annotations

import asyncio
import socket
import threading

import numpy as np
import pytest
from fastapi.testclient import TestClient

from inference_arena_amd.data.synthetic import encode_jpeg, synthetic_images
from inference_arena_amd.processing import extract_crop
from inference_arena_amd.processing.mobilenet_preprocess import crop_bounds
from inference_arena_amd.proto import inference_api as pb
from inference_arena_amd.server.device_transport import (DeviceClassifier, DeviceImageRing, ImageKey,
                                                         device_batch_request, group_by_image, is_device_request)
from inference_arena_amd.server.multipart import encode_multipart
from inference_arena_amd.server.service_backends import ClassifierBackend, DetectorBackend
from inference_arena_amd.utils.settings import Settings


class FakeDevice:
    """Device memory of the fake: IPC handle -> (base address, bytearray)."""

    def __init__(self):
        self.mem: dict[bytes, tuple[int, bytearray]] = {}
        self.opened: list[bytes] = []

    def open(self, handle: bytes) -> tuple[int, int]:
        self.opened.append(handle)
        base, buf = self.mem[handle]
        return base, len(buf)

    def resolve(self, ptr: int) -> tuple[bytearray, int]:
        for base, buf in self.mem.values():
            if base <= ptr < base + len(buf):
                return buf, ptr - base
        raise ValueError(f"unmapped device address {ptr:#x}")


class FakeIpcBuffer:
    def __init__(self, dev: FakeDevice, nbytes: int, tag: int):
        self.data = bytearray(nbytes)
        self._handle = bytes([tag]) * 64
        dev.mem[self._handle] = ((tag + 1) << 40, self.data)

    def handle(self) -> bytes:
        return self._handle

    def write(self, off: int, arr: np.ndarray) -> None:
        b = arr.tobytes()
        self.data[off: off + len(b)] = b


def fake_class(crop: np.ndarray) -> int:
    return int(crop.shape[0] % 1000)  # the FakeClassifier rule of test_microservices.py: crop height


class FakeFrameBackend:
    """Stands in for GpuFrameClassifier: reads each frame out of the fake device memory, cuts the crops with the
    crop-plan rule and 'classifies' them by height."""

    def __init__(self, dev: FakeDevice):
        self.dev = dev
        self.batches: list[int] = []
        self._results = {}
        self._lock = threading.Lock()
        self._slot = 0

    def submit(self, images, boxes) -> int:
        self.batches.append(len(images))
        ids, offs = [], [0]
        for (ptr, h, w, _device), bx in zip(images, boxes):
            buf, off = self.dev.resolve(ptr)
            frame = np.frombuffer(bytes(buf[off: off + h * w * 3]), np.uint8).reshape(h, w, 3)
            for b in bx:
                ids.append(fake_class(extract_crop(frame, b)))
            offs.append(len(ids))
        k = len(ids)
        res = {"crop_offset": np.array(offs, np.int32),
               "topk_idx": np.stack([np.array([c, 1, 2, 3, 4], np.int32) for c in ids]) if k else np.zeros((0, 5), np.int32),
               "topk_prob": np.tile(np.array([0.6, 0.2, 0.1, 0.05, 0.05], np.float32), (k, 1))}
        with self._lock:  # DeviceClassifier submits from up to ``inflight`` threads
            self._slot += 1
            slot = self._slot
            self._results[slot] = res
        return slot

    def collect(self, slot: int) -> dict:
        return self._results.pop(slot)


def test_ring_slots_offsets_and_backpressure():
    dev = FakeDevice()
    ring = DeviceImageRing(2, 64 * 64 * 3, device=3, buffer=FakeIpcBuffer(dev, 2 * 64 * 64 * 3, 7))
    a = np.full((10, 20, 3), 5, np.uint8)
    s0, r0 = ring.put(a)
    s1, r1 = ring.put(np.full((64, 64, 3), 9, np.uint8))
    assert {r0.offset, r1.offset} == {0, 64 * 64 * 3} and r0.offset == s0 * ring.slot_bytes
    assert (r0.height, r0.width, r0.device, r0.handle) == (10, 20, 3, bytes([7]) * 64)
    assert bytes(dev.mem[r0.handle][1][r0.offset: r0.offset + a.nbytes]) == a.tobytes()
    with pytest.raises(TimeoutError):  # both slots in flight
        ring.acquire(timeout=0.05)
    ring.release(s0)
    s2, r2 = ring.put(a)
    assert s2 == s0
    with pytest.raises(ValueError):
        ring.put(np.zeros((65, 64, 3), np.uint8))  # larger than a slot
    with pytest.raises(ValueError):
        ring.put(np.zeros((4, 4), np.uint8))


def test_handle_protocol_roundtrip_and_grouping():
    ref = pb.DeviceImageRef(handle=b"\x01" * 64, device=1, offset=3 << 32, height=480, width=640)
    boxes = [{"x1": 1, "y1": 2, "x2": 30, "y2": 40, "confidence": 0.9, "class_id": 5},
             {"x1": 0, "y1": 0, "x2": 640, "y2": 480, "confidence": 0.5, "class_id": 0}]
    wire = device_batch_request("rq", ref, boxes).SerializeToString()
    req = pb.BatchClassificationRequest.FromString(wire)
    assert [r.request_id for r in req.requests] == ["rq_0", "rq_1"]
    assert all(is_device_request(r) and r.image_crop == b"" for r in req.requests)
    # a second frame interleaved: grouping keeps first-seen order and request indices
    other = device_batch_request("o", pb.DeviceImageRef(handle=b"\x02" * 64, height=8, width=8), boxes[:1])
    mixed = [req.requests[0], other.requests[0], req.requests[1]]
    g = group_by_image(mixed)
    assert [k for k, _, _ in g] == [ImageKey(b"\x01" * 64, 1, 3 << 32, 480, 640), ImageKey(b"\x02" * 64, 0, 0, 8, 8)]
    assert g[0][2] == [0, 2] and g[1][2] == [1]
    np.testing.assert_array_equal(g[0][1], np.float32([[1, 2, 30, 40, 0.9, 5], [0, 0, 640, 480, 0.5, 0]]))
    assert g[0][1].dtype == np.float32
    # a reference peer parsing the arena request just skips field 100
    assert not is_device_request(pb.ClassificationRequest(request_id="x", image_crop=b"\x01"))


def test_device_classifier_batches_frames_and_maps_each_handle_once():
    dev = FakeDevice()
    rings = [DeviceImageRing(8, 32 * 32 * 3, buffer=FakeIpcBuffer(dev, 8 * 32 * 32 * 3, t)) for t in (1, 2)]
    be = FakeFrameBackend(dev)
    dc = DeviceClassifier(be, dev.open, max_batch=4, max_crops=6, max_delay_us=20000)
    frames = []
    for i in range(6):
        img = np.full((16 + i, 32, 3), i, np.uint8)
        _, ref = rings[i % 2].put(img)
        frames.append((ImageKey(ref.handle, 0, ref.offset, ref.height, ref.width),
                       np.array([[0, 0, 8, 4 + i, 0.9, 1], [0, 0, 32, 16 + i, 0.8, 2]], np.float32)))

    async def go():
        out = await asyncio.gather(*(dc.classify(k, b) for k, b in frames))
        dc.close()
        return out

    out = asyncio.run(go())
    for i, res in enumerate(out):
        assert [r[0][0] for r in res] == [4 + i, 16 + i]  # crop heights of this frame's boxes
        assert res[0][1][0] == pytest.approx(0.6)
    assert sum(be.batches) == 6 and max(be.batches) == 3  # 2 crops per frame, 6 crops per batch at most
    assert sorted(set(dev.opened)) == sorted({r.handle for r in rings}) and len(dev.opened) == 2


def test_device_classifier_failure_reaches_every_waiter():
    class Boom(FakeFrameBackend):
        def submit(self, images, boxes):
            raise RuntimeError("submit_device: batch exceeds the staging pool")

    dev = FakeDevice()
    ring = DeviceImageRing(2, 300, buffer=FakeIpcBuffer(dev, 600, 1))
    _, ref = ring.put(np.zeros((10, 10, 3), np.uint8))
    dc = DeviceClassifier(Boom(dev), dev.open, max_delay_us=1000)
    key = ImageKey(ref.handle, 0, ref.offset, 10, 10)

    async def go():
        r = await asyncio.gather(dc.classify(key, np.zeros((1, 6), np.float32)),
                                 dc.classify(key, np.zeros((2, 6), np.float32)), return_exceptions=True)
        dc.close()
        return r

    assert all(isinstance(e, RuntimeError) for e in asyncio.run(go()))


class FakeClassifier(ClassifierBackend):
    async def classify(self, crop):
        return (np.array([fake_class(crop), 1, 2, 3, 4], np.int32), np.array([5, 4, 3, 2, 1], np.float32),
                np.array([0.6, 0.2, 0.1, 0.05, 0.05], np.float32))


class FakeDetector(DetectorBackend):
    async def detect(self, image):
        h, w = image.shape[:2]
        return np.array([[0, 0, 10, 20, 0.9, 1], [5, 5, w, h, 0.7, 2], [3, 3, 3, 9, 0.6, 4],
                         [-4.5, 2.7, 33.9, 41.2, 0.5, 7]], np.float32), {}


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class ClassificationThread:
    def __init__(self, frames):
        from inference_arena_amd.server.classification_service import start_server

        self.port = _free_port()
        self.loop = asyncio.new_event_loop()
        ready = threading.Event()
        s = Settings(LOG_LEVEL="WARNING", HOST="127.0.0.1")

        async def boot():
            self.server, self.servicer, _ = await start_server(s, FakeClassifier(), port=self.port, frames=frames)
            ready.set()

        self.t = threading.Thread(target=lambda: (self.loop.run_until_complete(boot()), self.loop.run_forever()),
                                  daemon=True)
        self.t.start()
        assert ready.wait(20)

    def stop(self):
        asyncio.run_coroutine_threadsafe(self.server.stop(0), self.loop).result(10)
        self.loop.call_soon_threadsafe(self.servicer.close)
        self.loop.call_soon_threadsafe(self.loop.stop)
        self.t.join(10)


@pytest.mark.parametrize("transport", ["device", "raw"])
def test_predict_device_transport_matches_byte_transport(transport):
    """/predict over a live gRPC classification service: the device hand-off answers exactly what the byte path
    answers (same crops, cut on the receiving side), slots are returned, and the frame travels once."""
    from inference_arena_amd.server.detection_service import create_app

    dev = FakeDevice()
    be = FakeFrameBackend(dev)
    srv = ClassificationThread(DeviceClassifier(be, dev.open, max_delay_us=200))
    ring = DeviceImageRing(4, 640 * 640 * 3, buffer=FakeIpcBuffer(dev, 4 * 640 * 640 * 3, 9))
    try:
        s = Settings(LOG_LEVEL="WARNING", CLASSIFICATION_GRPC_ENDPOINT=f"127.0.0.1:{srv.port}",
                     ARENA_CROP_TRANSPORT=transport, ARENA_FANOUT="batch")
        img = synthetic_images(1, 5)[0]
        body, ctype = encode_multipart("file", encode_jpeg(img))
        app = create_app(s, detector=FakeDetector(), ring=ring if transport == "device" else None)
        with TestClient(app) as c:
            outs = [c.post("/predict", content=body, headers={"content-type": ctype}) for _ in range(3)]
        for r in outs:
            assert r.status_code == 200, r.text
        dets = outs[0].json()["detections"]
        h, w = img.shape[:2]
        expect = [20, h - 5, 1]
        x1, y1, x2, y2 = crop_bounds([-4.5, 2.7, 33.9, 41.2], h, w)
        expect.append((y2 - y1) % 1000)
        assert [d["classification"]["class_id"] for d in dets] == expect
        assert dets[3]["detection"]["x1"] == pytest.approx(-4.5)
        if transport == "device":
            assert sum(be.batches) == 3 and srv.servicer.n_errors == 0
            assert len(ring._free) == ring.slots  # every slot released after its answer
        else:
            assert be.batches == []
    finally:
        srv.stop()


def test_device_request_without_frame_classifier_is_an_in_band_error():
    srv = ClassificationThread(None)
    try:
        async def go():
            from inference_arena_amd.server.grpc_client import ClassificationClient

            cl = ClassificationClient(f"127.0.0.1:{srv.port}", transport="device")
            await cl.connect(10)
            ref = pb.DeviceImageRef(handle=b"\x05" * 64, height=4, width=4)
            out = await cl.classify_device("r", ref, [{"x1": 0, "y1": 0, "x2": 2, "y2": 2}])
            await cl.close()
            return out

        out = asyncio.run(go())
        assert len(out) == 1 and "not enabled" in out[0].error and out[0].request_id == "r_0"
    finally:
        srv.stop()


def test_device_classifier_rejects_out_of_range_references():
    """A frame reference outside the exported ring, or non-finite / huge boxes, is an in-band error before any
    device work (no out-of-bounds device reads from a bad DeviceImageRef)."""
    dev = FakeDevice()
    ring = DeviceImageRing(2, 300, buffer=FakeIpcBuffer(dev, 600, 4))
    _, ref = ring.put(np.zeros((10, 10, 3), np.uint8))
    be = FakeFrameBackend(dev)
    dc = DeviceClassifier(be, dev.open, max_delay_us=1000)
    ok = np.array([[0, 0, 5, 5, 0.9, 1]], np.float32)
    cases = [
        (ImageKey(ref.handle, 0, 500, 10, 10), ok),                 # 300 bytes at 500 > 600-byte ring
        (ImageKey(ref.handle, 0, -3, 10, 10), ok),                  # negative offset
        (ImageKey(ref.handle, 0, 0, 0, 10), ok),                    # empty frame
        (ImageKey(ref.handle, 0, 0, 10, 10), np.array([[np.nan, 0, 5, 5, 0.9, 1]], np.float32)),
        (ImageKey(ref.handle, 0, 0, 10, 10), np.array([[0, 0, 3e9, 5, 0.9, 1]], np.float32)),
    ]

    async def go():
        r = await asyncio.gather(*(dc.classify(k, b) for k, b in cases), dc.classify(ImageKey(ref.handle, 0, 0, 10, 10), ok),
                                 return_exceptions=True)
        dc.close()
        return r

    out = asyncio.run(go())
    assert all(isinstance(e, ValueError) for e in out[:-1]), out
    assert not isinstance(out[-1], BaseException) and be.batches == [1]  # only the valid frame reached the device


def test_device_classifier_drops_cancelled_waiters():
    dev = FakeDevice()
    ring = DeviceImageRing(2, 300, buffer=FakeIpcBuffer(dev, 600, 5))
    _, ref = ring.put(np.zeros((10, 10, 3), np.uint8))
    be = FakeFrameBackend(dev)
    dc = DeviceClassifier(be, dev.open, max_delay_us=50000)
    key = ImageKey(ref.handle, 0, 0, 10, 10)
    box = np.array([[0, 0, 5, 5, 0.9, 1]], np.float32)

    async def go():
        t1 = asyncio.ensure_future(dc.classify(key, box))
        t2 = asyncio.ensure_future(dc.classify(key, box))
        await asyncio.sleep(0.005)
        t1.cancel()  # the RPC's deadline fired while the batch was still filling
        r = await t2
        dc.close()
        return r

    assert len(asyncio.run(go())) == 1
    assert be.batches == [1]  # the cancelled waiter's frame never reached the device


def test_predict_exports_the_detector_frame_into_the_ring():
    """With an exporting detector (the GPU one copies its staged frame into the ring slot device to device), the
    detection service never uploads the frame again (no DeviceImageRing.put), and the answers are unchanged."""
    from inference_arena_amd.server.detection_service import create_app

    dev = FakeDevice()

    class ExportingDetector(FakeDetector):
        exports_frames = True

        def __init__(self):
            self.exports = 0

        async def detect(self, image, export_to=0):
            if export_to:
                buf, off = dev.resolve(export_to)
                b = np.ascontiguousarray(image).tobytes()
                buf[off: off + len(b)] = b
                self.exports += 1
            return await super().detect(image)

    class CountingRing(DeviceImageRing):
        puts = 0

        def put(self, image):
            CountingRing.puts += 1
            return super().put(image)

    be = FakeFrameBackend(dev)
    srv = ClassificationThread(DeviceClassifier(be, dev.open, max_delay_us=200))
    ring = CountingRing(4, 640 * 640 * 3, buffer=FakeIpcBuffer(dev, 4 * 640 * 640 * 3, 12))
    ring.buf.ptr = dev.mem[ring.handle][0]
    det = ExportingDetector()
    try:
        s = Settings(LOG_LEVEL="WARNING", CLASSIFICATION_GRPC_ENDPOINT=f"127.0.0.1:{srv.port}",
                     ARENA_CROP_TRANSPORT="device", ARENA_FANOUT="batch")
        img = synthetic_images(1, 6)[0]
        body, ctype = encode_multipart("file", encode_jpeg(img))
        with TestClient(create_app(s, detector=det, ring=ring)) as c:
            outs = [c.post("/predict", content=body, headers={"content-type": ctype}) for _ in range(3)]
        h = img.shape[0]
        for r in outs:
            assert r.status_code == 200, r.text
            assert [d["classification"]["class_id"] for d in r.json()["detections"]][:3] == [20, h - 5, 1]
        assert det.exports == 3 and CountingRing.puts == 0 and sum(be.batches) == 3
        assert len(ring._free) == ring.slots
    finally:
        srv.stop()


def test_predict_device_transport_with_the_split_decoder():
    """Device transport + an exporting detector with the split decoder (detect_bytes): the detection service never
    decodes the upload itself (only its header is probed for the frame size) and the answers are unchanged."""
    from inference_arena_amd.processing.transforms import load_image_from_bytes
    from inference_arena_amd.server.detection_service import create_app

    dev = FakeDevice()

    class SplitDetector(FakeDetector):
        exports_frames = True

        def __init__(self):
            self.bytes_calls = 0

        async def detect_bytes(self, data, decode, export_to=0):
            self.bytes_calls += 1
            image = load_image_from_bytes(data)  # stands in for the GPU reconstruction
            buf, off = dev.resolve(export_to)
            b = np.ascontiguousarray(image).tobytes()
            buf[off: off + len(b)] = b
            return await super().detect(image)

    be = FakeFrameBackend(dev)
    srv = ClassificationThread(DeviceClassifier(be, dev.open, max_delay_us=200))
    ring = DeviceImageRing(4, 640 * 640 * 3, buffer=FakeIpcBuffer(dev, 4 * 640 * 640 * 3, 13))
    ring.buf.ptr = dev.mem[ring.handle][0]
    det = SplitDetector()
    try:
        s = Settings(LOG_LEVEL="WARNING", CLASSIFICATION_GRPC_ENDPOINT=f"127.0.0.1:{srv.port}",
                     ARENA_CROP_TRANSPORT="device", ARENA_FANOUT="batch")
        img = synthetic_images(1, 8)[0]
        body, ctype = encode_multipart("file", encode_jpeg(img))
        app = create_app(s, detector=det, ring=ring)
        with TestClient(app) as c:
            outs = [c.post("/predict", content=body, headers={"content-type": ctype}) for _ in range(2)]
        h = img.shape[0]
        for r in outs:
            assert r.status_code == 200, r.text
            assert [d["classification"]["class_id"] for d in r.json()["detections"]][:3] == [20, h - 5, 1]
        assert det.bytes_calls == 2 and sum(be.batches) == 2 and len(ring._free) == ring.slots
    finally:
        srv.stop()
