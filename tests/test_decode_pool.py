"""Multi-process decode pool (server/decode_pool.py): pixels identical to load_image_from_bytes on every
transport path (slot, inline upload, oversize result), errors returned as text, slots recycled."""
from __future__ import annotations

import io
import threading

import numpy as np
import pytest
from PIL import Image

from inference_arena_amd.processing.transforms import decode_rgb, load_image_from_bytes
from inference_arena_amd.server.decode_pool import ProcessDecodePool


def _jpeg(h, w, seed, mode="RGB"):
    rng = np.random.default_rng(seed)
    arr = rng.integers(0, 255, (h, w, 3) if mode == "RGB" else (h, w), dtype=np.uint8)
    buf = io.BytesIO()
    Image.fromarray(arr, mode).save(buf, format="JPEG" if mode == "RGB" else "PNG", quality=90)
    return buf.getvalue()


def _run(pool, payloads):
    out, done = {}, threading.Semaphore(0)

    def cb(tag, view, err):
        out[tag] = (None if view is None else view.copy(), err)
        done.release()
    for i, p in enumerate(payloads):
        pool.submit(p, i, cb)
    for _ in payloads:
        assert done.acquire(timeout=60)
    return out


@pytest.fixture(scope="module")
def payloads():
    return [_jpeg(48 + 8 * i, 64 + 4 * i, i) for i in range(6)] + [_jpeg(40, 56, 99, mode="L")]


def test_decode_rgb_matches_loader(payloads):
    for p in payloads:
        h, w, px = decode_rgb(p)
        ref = load_image_from_bytes(p)
        assert ref.shape == (h, w, 3)
        assert np.array_equal(np.frombuffer(px, np.uint8).reshape(h, w, 3), ref)
    with pytest.raises(ValueError, match="Failed to decode image"):
        decode_rgb(b"")
    with pytest.raises(ValueError, match="Failed to decode image"):
        decode_rgb(b"not an image")


def test_pool_paths(payloads):
    # tiny in/out regions force the inline-upload and oversize-result paths for the larger images
    with ProcessDecodePool(workers=2, slots=3, slot_pixels=60 * 80, in_bytes=3000) as pool:
        data = payloads + [b"garbage", b""] + payloads
        out = _run(pool, data)
    for i, p in enumerate(data):
        view, err = out[i]
        if p in (b"garbage", b""):
            assert view is None and "Failed to decode image" in err
        else:
            assert err is None
            assert np.array_equal(view, load_image_from_bytes(p))


def _bomb_jpeg(h: int = 40000, w: int = 40000) -> bytes:
    """A valid 16x16 JPEG whose SOF0 header declares h x w pixels: a few hundred bytes that would decode to
    gigabytes (one such upload used to kill a decode worker)."""
    data = bytearray(_jpeg(16, 16, 5))
    i = data.index(b"\xff\xc0")  # baseline SOF0: marker, length(2), precision(1), height(2), width(2)
    data[i + 5:i + 7] = h.to_bytes(2, "big")
    data[i + 7:i + 9] = w.to_bytes(2, "big")
    return bytes(data)


def test_decode_rgb_rejects_decompression_bomb():
    from inference_arena_amd.processing.transforms import ImageTooLargeError

    with pytest.raises(ImageTooLargeError, match="image too large"):
        decode_rgb(_bomb_jpeg())
    with pytest.raises(ImageTooLargeError):
        load_image_from_bytes(_bomb_jpeg())


def test_pool_survives_bomb_and_dead_worker(payloads):
    """A bomb upload comes back as an error and the worker keeps serving; a worker killed from outside is
    replaced by the watchdog, and the pool keeps answering (no slot or callback is lost)."""
    import os
    import signal
    import time

    with ProcessDecodePool(workers=2, slots=8) as pool:
        out = _run(pool, [_bomb_jpeg(), payloads[0], _bomb_jpeg(30000, 5000), payloads[1]])
        assert out[0][0] is None and "image too large" in out[0][1]
        assert out[2][0] is None and "image too large" in out[2][1]
        np.testing.assert_array_equal(out[1][0], load_image_from_bytes(payloads[0]))
        assert out[3][1] is None
        os.kill(pool.procs[0].pid, signal.SIGKILL)
        t0 = time.time()
        while pool.respawned < 1 and time.time() - t0 < 30:
            time.sleep(0.1)
        assert pool.respawned == 1 and pool.dead_workers == 1
        out = _run(pool, payloads * 3)  # more uploads than slots: every slot came back
        assert all(err is None for _, err in out.values())
        for i, p in enumerate(payloads * 3):
            np.testing.assert_array_equal(out[i][0], load_image_from_bytes(p))
