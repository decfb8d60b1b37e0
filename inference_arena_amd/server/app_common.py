"""Pieces shared by the HTTP front-ends of all topologies.

* request-id + JSON logging per request (reference: architectures/*/app/
  main.py sets ``request_id_var`` from a uuid4 and logs endpoint / latency /
  detections / status_code);
* multipart ``file`` extraction and image decoding on a bounded thread pool
  (PIL releases the GIL while decoding, so decoding scales with cores instead
  of blocking the event loop);
* result -> ``PredictResponse`` conversion with the per-topology confidence
  semantics (raw top-1 logit for monolithic / gateway, softmax probability
  for microservices — the reference's behaviour);
* optional fault injection (``ARENA_FAULT_EVERY=k`` fails every k-th request)
  to exercise client/error paths.
"""
from __future__ import annotations

import asyncio
import itertools
import os
import logging
import time
import uuid
from concurrent.futures import ThreadPoolExecutor

import numpy as np
from fastapi import HTTPException, Request

from ..engine.pipeline import ImageResult
from ..processing import load_image_from_bytes
from ..utils.logging import request_id_var
from .multipart import MultipartError, parse_multipart
from .schemas import Classification, DetectionBox, DetectionWithClassification, PredictResponse

log = logging.getLogger("arena.server")


def probe_size(data: bytes) -> tuple[int, int]:
    """(height, width) of an encoded upload from its header alone (PIL's lazy open, no pixel decode); the
    errors of a failed decode: ValueError, TooLarge beyond ``max_image_pixels``."""
    import io

    from PIL import Image, UnidentifiedImageError

    from ..processing.transforms import max_image_pixels
    from .batching import TooLarge

    if not data:
        raise ValueError("Failed to decode image: empty payload")
    try:
        with Image.open(io.BytesIO(data)) as im:
            w, h = im.size
    except (UnidentifiedImageError, OSError, ValueError) as e:
        raise ValueError(f"Failed to decode image: {e}") from e
    if w * h > max_image_pixels():
        raise TooLarge(f"Failed to decode image: image too large ({w}x{h} pixels > {max_image_pixels()})")
    return h, w


class DecodePool:
    """Upload decode off the event loop.  ``procs`` > 0 (``ARENA_DECODE_PROCS``): spawned decode processes
    with shared-memory delivery (server/decode_pool.py; scales with cores, unlike PIL threads whose
    numpy conversion holds the GIL); otherwise a thread pool of ``threads``."""

    def __init__(self, threads: int = 8, procs: int | None = None):
        procs = int(os.environ.get("ARENA_DECODE_PROCS", "0")) if procs is None else int(procs)
        self.procs = None
        self.pool = None
        if procs > 0:
            from .decode_pool import ProcessDecodePool

            self.procs = ProcessDecodePool(workers=procs, slots=max(64, 8 * procs))
        else:
            self.pool = ThreadPoolExecutor(max_workers=max(1, threads), thread_name_prefix="decode")

    async def decode(self, data: bytes) -> np.ndarray:
        """Raises ``TooLarge`` (servers answer 413) for a header that declares more pixels than the decoder
        accepts (processing/transforms.py ImageTooLargeError), ``ValueError`` for any other decode failure."""
        from ..processing.transforms import ImageTooLargeError
        from .batching import TooLarge

        if self.procs is None:
            try:
                return await asyncio.get_running_loop().run_in_executor(self.pool, load_image_from_bytes, data)
            except ImageTooLargeError as e:
                raise TooLarge(str(e)) from e
        loop = asyncio.get_running_loop()
        fut: asyncio.Future = loop.create_future()

        def done(_tag, img, err):
            # runs on the pool's collector thread; the shared-memory slot is reused after return: copy out
            res = (None, err) if err is not None else (np.array(img), None)
            loop.call_soon_threadsafe(lambda: fut.done() or fut.set_result(res))

        await loop.run_in_executor(None, self.procs.submit, data, None, done)
        img, err = await fut
        if err is not None:
            raise TooLarge(err) if "image too large" in err else ValueError(err)
        return img

    def close(self) -> None:
        if self.pool is not None:
            self.pool.shutdown(wait=False)
        if self.procs is not None:
            self.procs.close()


async def read_upload(request: Request, field: str = "file") -> bytes:
    body = await request.body()
    ctype = request.headers.get("content-type", "")
    if ctype.lower().startswith("multipart/form-data"):
        try:
            parts = parse_multipart(body, ctype)
        except MultipartError as e:
            raise HTTPException(status_code=422, detail=str(e)) from e
        if field not in parts:
            raise HTTPException(status_code=422, detail=f"missing form field '{field}'")
        return parts[field][0]
    if body:
        return body  # raw image body (application/octet-stream, image/jpeg)
    raise HTTPException(status_code=422, detail="empty request body")


def to_response(rid: str, res: ImageResult, labels: list[str], timing: dict, confidence: str = "logit"
                ) -> PredictResponse:
    dets = []
    for i in range(len(res)):
        b = res.boxes[i]
        cid = int(res.topk_idx[i, 0]) if res.topk_idx.shape[0] > i else -1
        conf = float(res.topk_prob[i, 0] if confidence == "softmax" else res.topk_logit[i, 0]) if cid >= 0 else 0.0
        dets.append(DetectionWithClassification(
            detection=DetectionBox(x1=float(b[0]), y1=float(b[1]), x2=float(b[2]), y2=float(b[3]),
                                   confidence=float(res.scores[i]), class_id=int(res.classes[i])),
            classification=Classification(class_id=cid, class_name=labels[cid] if 0 <= cid < len(labels) else "",
                                          confidence=conf),
        ))
    return PredictResponse(request_id=rid, detections=dets, timing={k: float(v) for k, v in timing.items()})


class FaultInjector:
    """``ARENA_FAULT_EVERY=k`` fails every k-th request.  ``ARENA_FAULT_MODE=device`` makes the injected
    failure a device fault (a message starting with "HIP error", as ARENA_HIP_CHECK raises): the service
    then reports itself unhealthy and a supervised replica exits so its launcher starts a fresh process."""

    def __init__(self, every: int = 0, mode: str | None = None):
        self.every = int(every)
        self.mode = (mode if mode is not None else os.environ.get("ARENA_FAULT_MODE", "request")).lower()
        self._n = itertools.count(1)
        self.device_error: str | None = None

    def check(self) -> None:
        if self.every > 0 and next(self._n) % self.every == 0:
            if self.mode == "device":
                self.device_error = "HIP error (injected by ARENA_FAULT_MODE=device)"
                raise RuntimeError(self.device_error)
            raise RuntimeError("injected fault (ARENA_FAULT_EVERY)")


def device_fault(state: dict) -> str | None:
    """The first device fault of a service (its backend's or an injected one), else None."""
    be = state.get("backend") or state.get("detector")
    err = getattr(be, "device_error", None) if be is not None else None
    f = state.get("faults")
    return err or (f.device_error if f is not None else None)


def new_request_id() -> str:
    rid = str(uuid.uuid4())
    request_id_var.set(rid)
    return rid


class Timer:
    def __init__(self):
        self.t0 = time.perf_counter()

    def ms(self) -> float:
        return (time.perf_counter() - self.t0) * 1e3
