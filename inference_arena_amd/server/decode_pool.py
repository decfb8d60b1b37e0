"""Multi-process JPEG decode pool with shared-memory delivery.

The reference decodes every upload on the request thread (cv2.imdecode in
src/shared/processing/transforms.py:77-110; PIL in
architectures/microservices/classification/app/servicer.py:65-76).  At GPU
request rates the decode is the host's largest per-request cost (about
1.5-3 ms of CPU per COCO-sized JPEG), and a thread pool does not scale: the
PIL -> numpy conversion holds the GIL (measured here: 8 threads decode only
1.4x faster than one).  This pool decodes in ``workers`` separate processes
(spawned, never forked: the parent may already hold GPU state) with the same
``load_image_from_bytes`` as every other path, writes the RGB pixels into a
slot of one shared-memory segment and hands the parent a zero-copy numpy view
of the slot.  The parent passes the view straight to the native batcher
(whose ``enqueue`` copies it) and the slot returns to the free list.

Images larger than a slot travel back pickled through the result queue
(correct, just slower); undecodable uploads come back as an error string.
"""
from __future__ import annotations

import multiprocessing as mp
import os
import queue
import threading
from multiprocessing import shared_memory
from typing import Callable

import numpy as np

DecodeCallback = Callable[[object, "np.ndarray | None", "str | None"], None]


def _worker(shm_name: str, slot_bytes: int, tasks, results) -> None:  # pragma: no cover - runs in a child
    from ..processing.transforms import load_image_from_bytes

    shm = shared_memory.SharedMemory(name=shm_name)
    try:
        while True:
            t = tasks.get()
            if t is None:
                return
            tag, slot, data = t
            try:
                img = load_image_from_bytes(data)
            except Exception as e:  # noqa: BLE001 - reported to the caller
                results.put((tag, slot, 0, 0, None, str(e)))
                continue
            h, w = img.shape[:2]
            if h * w * 3 <= slot_bytes:
                view = np.ndarray((h, w, 3), dtype=np.uint8, buffer=shm.buf, offset=slot * slot_bytes)
                view[...] = img
                del view
                results.put((tag, slot, h, w, None, None))
            else:
                results.put((tag, slot, h, w, np.ascontiguousarray(img).tobytes(), None))
    finally:
        shm.close()


class ProcessDecodePool:
    """``submit(jpeg_bytes, tag, callback)``; ``callback(tag, rgb_view_or_None, error_or_None)`` runs on the
    pool's collector thread and must consume the view before returning (the slot is reused afterwards)."""

    def __init__(self, workers: int | None = None, slots: int = 256, slot_pixels: int = 1024 * 1024):
        self.workers = max(1, int(workers or min(16, os.cpu_count() or 4)))
        self.slots = int(slots)
        self.slot_bytes = int(slot_pixels) * 3
        self.shm = shared_memory.SharedMemory(create=True, size=self.slots * self.slot_bytes)
        ctx = mp.get_context("spawn")
        self.tasks = ctx.Queue()
        self.results = ctx.Queue()
        self.procs = [ctx.Process(target=_worker, args=(self.shm.name, self.slot_bytes, self.tasks, self.results),
                                  daemon=True, name=f"arena-decode-{i}") for i in range(self.workers)]
        for p in self.procs:
            p.start()
        self._free: queue.SimpleQueue = queue.SimpleQueue()
        for s in range(self.slots):
            self._free.put(s)
        self._cbs: dict[int, tuple[object, DecodeCallback]] = {}
        self._lock = threading.Lock()
        self._seq = 0
        self._closed = False
        self._collector = threading.Thread(target=self._collect, name="arena-decode-collector", daemon=True)
        self._collector.start()

    def submit(self, data: bytes, tag, callback: DecodeCallback) -> None:
        """Queue one encoded image; blocks while every slot is in use."""
        if self._closed:
            raise RuntimeError("decode pool is closed")
        slot = self._free.get()
        with self._lock:
            self._seq += 1
            key = self._seq
            self._cbs[key] = (tag, callback)
        self.tasks.put((key, slot, data))

    def _collect(self) -> None:
        while True:
            r = self.results.get()
            if r is None:
                return
            key, slot, h, w, payload, err = r
            with self._lock:
                tag, cb = self._cbs.pop(key)
            try:
                if err is not None:
                    cb(tag, None, err)
                elif payload is not None:
                    cb(tag, np.frombuffer(payload, dtype=np.uint8).reshape(h, w, 3), None)
                else:
                    cb(tag, np.ndarray((h, w, 3), dtype=np.uint8, buffer=self.shm.buf,
                                       offset=slot * self.slot_bytes), None)
            except Exception as e:  # noqa: BLE001 - a failing consumer must not stop the pool
                import sys

                print(f"decode pool callback failed: {e!r}", file=sys.stderr)
            finally:
                self._free.put(slot)

    def close(self) -> None:
        if self._closed:
            return
        self._closed = True
        for _ in self.procs:
            self.tasks.put(None)
        for p in self.procs:
            p.join(timeout=5)
            if p.is_alive():
                p.terminate()
        self.results.put(None)
        self._collector.join(timeout=5)
        try:
            self.shm.close()
            self.shm.unlink()
        except (FileNotFoundError, BufferError):
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
