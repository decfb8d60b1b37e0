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
