"""Multi-process JPEG decode pool with shared-memory transport both ways.

The reference decodes every upload on the request thread (cv2.imdecode in
src/shared/processing/transforms.py:77-110; PIL in
architectures/microservices/classification/app/servicer.py:65-76).  At GPU
request rates the decode is the host's largest per-request cost (about
1-3 ms of CPU per COCO-sized JPEG), and a thread pool does not scale: the
PIL -> numpy conversion holds the GIL (measured here: 8 threads decode only
1.4x faster than one).  This pool decodes in ``workers`` separate processes
(spawned, never forked: the parent may already hold GPU state) with the same
decoder as every other path (``processing.transforms.decode_rgb``).

Transport is built so the parent does O(1) Python work per image and never
pickles a payload (the first version moved JPEG bytes and results through
``multiprocessing.Queue``s and saturated at ~6k decodes/s on a 16-core share,
profiles/r2_decode_rate.log, with the parent's pickling and queue locks as
the limit):

* one shared-memory segment of ``slots`` slots; a slot holds the upload
  (``in_bytes``) followed by room for its decoded RGB pixels (``slot_pixels``);
* the parent copies the upload into the slot and sends a 16-byte task record
  on the chosen worker's own pipe (least outstanding work first); uploads
  larger than ``in_bytes`` travel inline on that pipe instead;
* workers decode straight from the slot, write the packed RGB pixels into it
  and post a 32-byte completion record on ONE shared result pipe (writes of
  <= PIPE_BUF bytes are atomic, so no lock is needed across workers);
* the collector thread reads completion records in bulk and hands the callback
  a zero-copy numpy view of the slot; the slot is freed when the callback
  returns.  Images too large for a slot follow their record on the worker's
  result connection; undecodable uploads return their error text in the slot.
"""
from __future__ import annotations

import multiprocessing as mp
import os
import queue
import struct
import threading
from multiprocessing import shared_memory
from typing import Callable

import numpy as np

DecodeCallback = Callable[[object, "np.ndarray | None", "str | None"], None]

_TASK = struct.Struct("<qii")      # key, slot, payload length (-1: payload inline after the record)
_DONE = struct.Struct("<qiiiiq")   # key, slot, h, w, status, aux
_OK, _ERR, _BIG = 0, 1, 2          # pixels in slot / error text in slot (aux = length) / pixels on worker conn


def _worker(idx: int, shm_name: str, in_bytes: int, slot_bytes: int, tasks, results_w, big_w,
            cpus=None) -> None:  # pragma: no cover - runs in a child
    from ..processing.transforms import decode_rgb

    if cpus:  # this rank's host-CPU share (parallel/affinity.py), set inside the child
        try:
            os.sched_setaffinity(0, cpus)
        except OSError:
            pass

    shm = shared_memory.SharedMemory(name=shm_name)
    buf = shm.buf
    rfd = results_w.fileno()
    stride = in_bytes + slot_bytes
    try:
        while True:
            msg = tasks.recv_bytes()
            if not msg:
                return
            key, slot, n = _TASK.unpack_from(msg)
            base = slot * stride
            data = msg[_TASK.size:] if n < 0 else buf[base:base + n]
            try:
                h, w, px = decode_rgb(data)
            except Exception as e:  # noqa: BLE001 - any decoder failure (MemoryError included) is this upload's
                text = (str(e) or type(e).__name__).encode()[:slot_bytes]
                buf[base + in_bytes:base + in_bytes + len(text)] = text
                os.write(rfd, _DONE.pack(key, slot, 0, 0, _ERR, len(text)))
                continue
            finally:
                if n >= 0:
                    del data  # release the memoryview of the slot
            if len(px) <= slot_bytes:
                buf[base + in_bytes:base + in_bytes + len(px)] = px
                os.write(rfd, _DONE.pack(key, slot, h, w, _OK, 0))
            else:
                os.write(rfd, _DONE.pack(key, slot, h, w, _BIG, idx))
                big_w.send_bytes(px)
    finally:
        del buf
        shm.close()


def prestart() -> None:
    """Start the multiprocessing fork server now.  Call this before the process initialises the GPU: decode
    workers created later (pools built after the engines, replacements for dead workers) are then forked from
    that GPU-free server instead of being fork+exec'd from a process holding GPU state."""
    from multiprocessing import forkserver

    forkserver.ensure_running()


class ProcessDecodePool:
    """``submit(jpeg_bytes, tag, callback)``; ``callback(tag, rgb_view_or_None, error_or_None)`` runs on the
    pool's collector thread and must consume the view before returning (the slot is reused afterwards)."""

    def __init__(self, workers: int | None = None, slots: int = 256, slot_pixels: int = 1024 * 1024,
                 in_bytes: int = 1 << 20, native: bool = False, cpus: list[int] | None = None):
        """``native=True``: the parent side of the transport is driven by C++ (the native HTTP front end,
        csrc/runtime/http_front.h) through ``native_channel()``; no collector thread runs here."""
        self.workers = max(1, int(workers or min(16, os.cpu_count() or 4)))
        self.slots = int(slots)
        self.slot_bytes = int(slot_pixels) * 3
        self.in_bytes = int(in_bytes)
        self._stride = self.in_bytes + self.slot_bytes
        self.cpus = list(cpus) if cpus else None
        self.shm = shared_memory.SharedMemory(create=True, size=self.slots * self._stride)
        # forkserver, not spawn: the fork server starts here (before this process touches the GPU) and every
        # worker, including a replacement spawned after a worker died, is forked from it, never fork+exec'd from
        # a process that holds GPU state
        ctx = mp.get_context("forkserver")
        self._ctx = ctx
        self._res_r, self._res_w = ctx.Pipe(duplex=False)
        self._tasks, self._big, self.procs = [], [], []
        for i in range(self.workers):
            p, tw, br = self._spawn(i)
            self._tasks.append(tw)
            self._big.append(br)
            self.procs.append(p)
        self._send_locks = [threading.Lock() for _ in range(self.workers)]
        self._load = [0] * self.workers
        self._free: queue.SimpleQueue = queue.SimpleQueue()
        for s in range(self.slots):
            self._free.put(s)
        self._cbs: dict[int, tuple[object, DecodeCallback, int, int]] = {}  # key -> (tag, callback, worker, slot)
        self._handled_dead: set[int] = set()
        self.dead_workers = 0      # workers that died (native mode: the owner restarts the process)
        self.respawned = 0
        self._lock = threading.Lock()
        self._seq = 0
        self._closed = False
        self.native = bool(native)
        self._native_view = None
        self._collector = None
        if not self.native:
            self._collector = threading.Thread(target=self._collect, name="arena-decode-collector", daemon=True)
            self._collector.start()
        self._watcher = threading.Thread(target=self._watch, name="arena-decode-watchdog", daemon=True)
        self._watcher.start()

    def _spawn(self, i: int):
        tr, tw = self._ctx.Pipe(duplex=False)
        br, bw = self._ctx.Pipe(duplex=False)
        p = self._ctx.Process(target=_worker, args=(i, self.shm.name, self.in_bytes, self.slot_bytes, tr,
                                                    self._res_w, bw, self.cpus), daemon=True,
                              name=f"arena-decode-{i}")
        p.start()
        tr.close()
        bw.close()
        return p, tw, br

    def _watch(self) -> None:
        """A worker that died (killed, or a crash in the decoder library) would leave its pending uploads
        unanswered and their slots taken forever.  Python mode: fail those uploads, free their slots and
        spawn a replacement worker.  Native mode (the C++ front end owns the pipes): count the death; the
        owner leaves rotation and exits non-zero so its supervisor restarts the process
        (server/native_front.py)."""
        import time

        while not self._closed:
            time.sleep(0.2)
            for i, proc in enumerate(list(self.procs)):
                if self._closed or proc.is_alive() or (self.native and i in self._handled_dead):
                    continue
                self._worker_died(i)

    def _worker_died(self, i: int) -> None:
        if self.native:
            self._handled_dead.add(i)
            self.dead_workers += 1
            return
        with self._send_locks[i]:
            if self._closed or self.procs[i].is_alive():
                return
            self.dead_workers += 1
            with self._lock:
                failed = [(k, self._cbs.pop(k)) for k in [k for k, v in self._cbs.items() if v[2] == i]]
                self._load[i] = 0
            for c in (self._tasks[i], self._big[i]):
                try:
                    c.close()
                except OSError:
                    pass
            self.procs[i], self._tasks[i], self._big[i] = self._spawn(i)
            self.respawned += 1
        for _key, (tag, cb, _w, slot) in failed:
            try:
                cb(tag, None, "Failed to decode image: decode worker died")
            except Exception:  # noqa: BLE001 - a failing consumer must not stop the pool
                pass
            finally:
                self._free.put(slot)

    def to_python_mode(self) -> None:
        """Hand a native-mode pool back to Python (``submit``): call after the native driver stopped reading the
        completion pipe (HttpFrontEnd.stop()); the same worker processes then serve Python callers."""
        if not self.native:
            return
        self.native = False
        self._handled_dead.clear()
        self._collector = threading.Thread(target=self._collect, name="arena-decode-collector", daemon=True)
        self._collector.start()

    def native_channel(self) -> dict:
        """Shared-memory address, geometry and pipe descriptors for a native driver (see __init__)."""
        import ctypes

        if not self.native:
            raise RuntimeError("native_channel() needs ProcessDecodePool(native=True)")
        if self._native_view is None:
            self._native_view = ctypes.c_char.from_buffer(self.shm.buf)
        return {"shm_addr": ctypes.addressof(self._native_view), "stride": self._stride, "in_bytes": self.in_bytes,
                "slot_bytes": self.slot_bytes, "slots": self.slots,
                "task_fds": [c.fileno() for c in self._tasks], "big_fds": [c.fileno() for c in self._big],
                "result_fd": self._res_r.fileno(), "result_wfd": self._res_w.fileno()}

    def submit(self, data: bytes, tag, callback: DecodeCallback) -> None:
        """Queue one encoded image; blocks while every slot is in use."""
        if self._closed:
            raise RuntimeError("decode pool is closed")
        if self.native:
            raise RuntimeError("a native decode pool is driven through native_channel()")
        slot = self._free.get()
        n = len(data)
        if n <= self.in_bytes:
            base = slot * self._stride
            self.shm.buf[base:base + n] = data
        with self._lock:
            self._seq += 1
            key = self._seq
            w = min(range(self.workers), key=self._load.__getitem__)
        # registration and send under the worker's send lock: the watchdog fails a dead worker's keys and
        # replaces its pipe under the same lock, so a key is never sent to a worker it was not failed for
        with self._send_locks[w]:
            with self._lock:
                self._load[w] += 1
                self._cbs[key] = (tag, callback, w, slot)
            msg = _TASK.pack(key, slot, n) if n <= self.in_bytes else _TASK.pack(key, slot, -1) + bytes(data)
            try:
                self._tasks[w].send_bytes(msg)
                return
            except OSError:  # the worker died: answer this upload now; the watchdog replaces the worker
                with self._lock:
                    entry = self._cbs.pop(key, None)
                    self._load[w] -= 1
        if entry is not None:
            try:
                callback(tag, None, "Failed to decode image: decode worker unavailable")
            finally:
                self._free.put(slot)

    def _collect(self) -> None:
        fd = self._res_r.fileno()
        pending = b""
        rec = _DONE.size
        while True:
            chunk = os.read(fd, 64 * rec)
            if not chunk:
                return
            pending += chunk
            full = len(pending) - len(pending) % rec
            for off in range(0, full, rec):
                key, slot, h, w, status, aux = _DONE.unpack_from(pending, off)
                if key < 0:
                    return
                self._complete(key, slot, h, w, status, aux)
            pending = pending[full:]

    def _complete(self, key, slot, h, w, status, aux) -> None:
        with self._lock:
            entry = self._cbs.pop(key, None)
            if entry is None:  # already failed by the watchdog (its worker died after posting): slot freed there
                return
            tag, cb, worker, _ = entry
            self._load[worker] -= 1
        out = slot * self._stride + self.in_bytes
        try:
            if status == _ERR:
                cb(tag, None, bytes(self.shm.buf[out:out + aux]).decode(errors="replace"))
            elif status == _BIG:
                try:
                    px = self._big[aux].recv_bytes()
                except (EOFError, OSError):
                    cb(tag, None, "Failed to decode image: decode worker died")
                    return
                cb(tag, np.frombuffer(px, dtype=np.uint8).reshape(h, w, 3), None)
            else:
                cb(tag, np.ndarray((h, w, 3), dtype=np.uint8, buffer=self.shm.buf, offset=out), None)
        except Exception as e:  # noqa: BLE001 - a failing consumer must not stop the pool
            import sys

            print(f"decode pool callback failed: {e!r}", file=sys.stderr)
        finally:
            self._free.put(slot)

    def close(self) -> None:
        if self._closed:
            return
        self._closed = True
        for w, conn in enumerate(self._tasks):
            try:
                with self._send_locks[w]:
                    conn.send_bytes(b"")
            except OSError:
                pass
        for p in self.procs:
            p.join(timeout=5)
            if p.is_alive():
                p.terminate()
        if self._collector is not None:
            os.write(self._res_w.fileno(), _DONE.pack(-1, 0, 0, 0, 0, 0))
            self._collector.join(timeout=5)
        self._native_view = None
        for c in self._tasks + self._big + [self._res_r, self._res_w]:
            c.close()
        try:
            self.shm.close()
            self.shm.unlink()
        except (FileNotFoundError, BufferError):
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
