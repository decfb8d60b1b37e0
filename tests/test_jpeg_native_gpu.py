"""Device half of the split JPEG decoder (csrc/kernels/jpeg_idct.hip) on the GPU.

* the reconstruction kernels against the host reference (the same integer arithmetic, kernels/jpeg_math.h)
  and against PIL — bit-exact over qualities, chroma samplings, grayscale and odd sizes;
* the executor's JPEG input path (Executor.submit with split-decoded uploads: coefficients DMA'd into the
  staging pool, reconstructed before the program) against the same pipeline fed PIL-decoded pixels: the
  detections and classifications must be identical, because the pixels are;
* the native HTTP front end with the split decoder over the GPU engine against the PIL decode pool.
"""
from __future__ import annotations

import io
import json

import numpy as np
import pytest
from PIL import Image

from inference_arena_amd.ops import native

pytestmark = pytest.mark.gpu


def _enc(arr, **kw) -> bytes:
    b = io.BytesIO()
    Image.fromarray(arr).save(b, "JPEG", **kw)
    return b.getvalue()


def _pil(data: bytes) -> np.ndarray:
    with Image.open(io.BytesIO(data)) as im:
        return np.asarray(im.convert("RGB"))


def _frames():
    from inference_arena_amd.data.synthetic import synthetic_images

    imgs = synthetic_images(6, 31) + synthetic_images(2, 32, hw=(333, 500)) + synthetic_images(2, 33, hw=(640, 427))
    rng = np.random.default_rng(5)
    imgs.append((rng.random((37, 53, 3)) * 255).astype(np.uint8))
    imgs.append((rng.random((41, 66, 3)) * 255).astype(np.uint8))  # width 2 mod 4 (the colour kernel's quads)
    return imgs


@pytest.mark.parametrize("subsampling", [0, 1, 2])
def test_device_reconstruction_is_bit_exact(device, subsampling):
    C = native()
    uploads = [_enc(im, quality=q, subsampling=subsampling) for im, q in zip(_frames(), [90, 95, 75, 100, 50] * 4)]
    gray = np.asarray(Image.fromarray(_frames()[0]).convert("L"))
    uploads.append(_enc(gray, quality=90))
    uploads.append(_enc(_frames()[1], quality=85, subsampling=subsampling, restart_marker_blocks=5))
    got = C.jpeg_decode_device(uploads, 0)
    for i, (data, rgb) in enumerate(zip(uploads, got)):
        st, err, host = C.jpeg_decode_host(data)
        assert st == "ok", err
        np.testing.assert_array_equal(rgb, host, err_msg=f"upload {i}: device vs host reference")
        np.testing.assert_array_equal(rgb, _pil(data), err_msg=f"upload {i}: device vs PIL")


@pytest.fixture(scope="module")
def fp32_pipe():
    import torch

    from inference_arena_amd.engine.pipeline import GpuPipeline
    from inference_arena_amd.models.zoo import make_mobilenet, make_yolo

    if not torch.cuda.is_available():
        pytest.skip("no GPU visible")
    return GpuPipeline(make_yolo(0, cls_shift=-20.0), make_mobilenet(1), device=0, buckets=[1, 8, 16], dtype="fp32")


def test_executor_jpeg_inputs_match_decoded_pixels(fp32_pipe):
    """Executor.run on split-decoded uploads == Executor.run on PIL-decoded frames (mixed batches too)."""
    imgs = _frames()
    uploads = [_enc(im, quality=90) for im in imgs]
    pixels = [_pil(u) for u in uploads]
    ex = fp32_pipe.ex
    a = ex.run(uploads[:8])
    b = ex.run(pixels[:8])
    mixed = ex.run([uploads[8], pixels[9], uploads[10], pixels[0]])
    ref = ex.run([pixels[8], pixels[9], pixels[10], pixels[0]])
    for x, y in ((a, b), (mixed, ref)):
        assert list(x["det_count"]) == list(y["det_count"])
        for k in ("det", "topk_idx", "topk_logit"):
            np.testing.assert_array_equal(np.asarray(x[k]), np.asarray(y[k]), err_msg=k)
    assert sum(b["det_count"]) > 0  # the comparison saw detections and crops


def test_native_front_split_decode_matches_pil_pool(fp32_pipe):
    """/predict through the native front end: split decoder (host Huffman + GPU reconstruction) vs every upload
    through the PIL decode processes — the same detections and classifications."""
    import http.client

    from inference_arena_amd.labels import load_labels
    from inference_arena_amd.server.native_front import NativeFrontEnd

    C = native()
    uploads = [_enc(im, quality=90) for im in _frames()[:6]]
    bnd = "b0undary"

    def post(port, data):
        body = (f"--{bnd}\r\nContent-Disposition: form-data; name=\"file\"; filename=\"x.jpg\"\r\n"
                f"Content-Type: image/jpeg\r\n\r\n").encode() + data + f"\r\n--{bnd}--\r\n".encode()
        c = http.client.HTTPConnection("127.0.0.1", port, timeout=60)
        c.request("POST", "/predict", body=body, headers={"Content-Type": f"multipart/form-data; boundary={bnd}"})
        r = c.getresponse()
        out = (r.status, json.loads(r.read()))
        c.close()
        return out

    answers = {}
    for threads in (4, 0):
        batcher = C.DynamicBatcher([fp32_pipe.ex], {"max_batch": 16, "max_queue_delay_us": 200})
        fe = NativeFrontEnd(batcher, load_labels(None), port=0, host="127.0.0.1", io_threads=2, decode_procs=2,
                            slots=16, decode_threads=threads)
        try:
            answers[threads] = [post(fe.port, u) for u in uploads]
            st = fe.stats()
            assert st["native_decoded"] == (len(uploads) if threads else 0)
            assert st["fallback_decoded"] == (0 if threads else len(uploads))
        finally:
            fe.close()
            batcher.shutdown()
    for (s1, d1), (s2, d2) in zip(answers[4], answers[0]):
        assert s1 == s2 == 200
        strip = [(d["detection"], d["classification"]) for d in d1["detections"]]
        assert strip == [(d["detection"], d["classification"]) for d in d2["detections"]]
