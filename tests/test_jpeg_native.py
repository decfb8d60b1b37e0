"""Host half of the split JPEG decoder (csrc/runtime/jpeg_decode.h) on CPU.

The reference decodes uploads with cv2 / PIL (src/shared/processing/transforms.py:77-110; PIL for arm B,
architectures/microservices/classification/app/servicer.py:65-76).  The split decoder must produce exactly the
pixels PIL produces, so every detection / classification downstream is unchanged: the host reference
reconstruction (``jpeg_decode_host``, the same integer arithmetic the GPU kernels run, kernels/jpeg_math.h) is
compared bit for bit with PIL over qualities, chroma samplings, grayscale, odd sizes and restart intervals;
formats it does not cover are reported as unsupported (the server sends them to the PIL pool) and broken files
as corrupt with PIL's messages."""
from __future__ import annotations

import io

import numpy as np
import pytest
from PIL import Image

from inference_arena_amd.ops import native


def _enc(arr, **kw) -> bytes:
    b = io.BytesIO()
    Image.fromarray(arr).save(b, "JPEG", **kw)
    return b.getvalue()


def _pil(data: bytes) -> np.ndarray:
    with Image.open(io.BytesIO(data)) as im:
        return np.asarray(im.convert("RGB"))


def _scene(h, w, seed=0):
    """A natural-ish frame: smooth gradients + blobs + noise (every DCT frequency band populated)."""
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w].astype(np.float32)
    img = np.stack([x / max(w, 1) * 200, y / max(h, 1) * 180, (x + y) / max(h + w, 1) * 150], -1)
    for _ in range(6):
        cy, cx, r = rng.uniform(0, h), rng.uniform(0, w), rng.uniform(3, max(4, min(h, w) / 3))
        img += (((y - cy) ** 2 + (x - cx) ** 2) < r * r)[..., None] * rng.uniform(-90, 90, 3)
    img += rng.normal(0, 12, img.shape)
    return np.clip(img, 0, 255).astype(np.uint8)


@pytest.mark.parametrize("quality", [50, 75, 90, 95, 100])
@pytest.mark.parametrize("subsampling", [0, 1, 2])  # 4:4:4, 4:2:2, 4:2:0
def test_bit_exact_with_pil(quality, subsampling):
    C = native()
    for i, (h, w) in enumerate([(427, 640), (480, 640), (37, 53), (16, 16), (9, 7), (101, 3)]):
        data = _enc(_scene(h, w, i), quality=quality, subsampling=subsampling)
        st, err, rgb = C.jpeg_decode_host(data)
        if subsampling and w <= 4:  # chroma narrower than 3 samples: libjpeg box-upsamples -> PIL fallback
            assert st == "unsupported"
            continue
        assert st == "ok", err
        np.testing.assert_array_equal(rgb, _pil(data))


@pytest.mark.parametrize("blocks", [1, 3, 7])
def test_restart_intervals_and_grayscale(blocks):
    C = native()
    img = _scene(120, 170, blocks)
    for arr in (img, np.asarray(Image.fromarray(img).convert("L"))):
        data = _enc(arr, quality=88, restart_marker_blocks=blocks)
        assert b"\xff\xdd" in data
        st, err, rgb = C.jpeg_decode_host(data)
        assert st == "ok", err
        np.testing.assert_array_equal(rgb, _pil(data))


def test_curated_workload_is_bit_exact():
    """The bench's own uploads (curated synthetic frames, JPEG q90)."""
    from inference_arena_amd.data.synthetic import encode_jpeg, synthetic_images

    C = native()
    for img in synthetic_images(12, 5):
        data = encode_jpeg(img, 90)
        st, err, rgb = C.jpeg_decode_host(data)
        assert st == "ok", err
        np.testing.assert_array_equal(rgb, _pil(data))


def test_coefficient_layout():
    C = native()
    data = _enc(_scene(40, 56), quality=90, subsampling=2)
    d = C.jpeg_coefs(data)
    assert d["status"] == "ok" and (d["width"], d["height"], d["layout"]) == (56, 40, 3)
    y, cb, cr = d["comps"]
    assert (y["h"], y["v"], cb["h"], cb["v"]) == (2, 2, 1, 1)
    assert (y["bw"], y["bh"]) == (8, 6) and (cb["bw"], cb["bh"]) == (4, 3)  # MCU grid 4 x 3 of 16x16
    assert (cb["cw"], cb["ch"]) == (28, 20)
    assert d["coef_count"] == (48 + 12 + 12) * 64 == len(d["coef"])
    assert cb["coef_off"] == 48 * 64 and cr["coef_off"] == 60 * 64


def test_unsupported_formats_go_to_the_fallback():
    C = native()
    img = _scene(64, 64)
    cases = {
        "progressive": _enc(img, quality=90, progressive=True),
    }
    b = io.BytesIO()
    Image.fromarray(img).convert("CMYK").save(b, "JPEG")
    cases["cmyk"] = b.getvalue()
    b = io.BytesIO()
    Image.fromarray(img).save(b, "PNG")
    cases["png"] = b.getvalue()
    for name, data in cases.items():
        st, err, rgb = C.jpeg_decode_host(data)
        assert st == "unsupported" and rgb is None, (name, st, err)


def test_corrupt_and_oversized_inputs():
    C = native()
    good = _enc(_scene(64, 80), quality=90)
    st, err, _ = C.jpeg_decode_host(good[: len(good) // 2])  # cut inside the scan
    assert st == "corrupt" and "truncated" in err
    with pytest.raises(OSError):  # PIL agrees that this upload is broken
        _pil(good[: len(good) // 2])
    st, err, _ = C.jpeg_decode_host(good[:30])  # cut inside the headers
    assert st == "corrupt"
    st, err, _ = C.jpeg_decode_host(good, max_pixels=64 * 80 - 1)
    assert st == "corrupt" and "image too large" in err
    # a scan cut short by a marker decodes (libjpeg warns; PIL returns the image)
    sos = good.rfind(b"\xff\xda")
    cut = good[: sos + 40] + b"\xff\xd9"
    st, err, rgb = C.jpeg_decode_host(cut)
    assert st == "ok", err
    np.testing.assert_array_equal(rgb, _pil(cut))
    rng = np.random.default_rng(3)
    for _ in range(200):  # fuzz: random byte flips never crash the decoder
        bad = bytearray(good)
        for k in rng.integers(2, len(bad), 8):
            bad[k] = int(rng.integers(0, 256))
        st, _, _ = C.jpeg_decode_host(bytes(bad))
        assert st in ("ok", "corrupt", "unsupported")


@pytest.mark.parametrize("jpeg_device", [True, False])
def test_ingest_matches_pil_decode_and_falls_back(jpeg_device):
    """csrc/runtime/jpeg_ingest.h behind AsyncBatcher.run_jpeg (the model server's IMAGE_BYTES path): the same
    answer as the PIL-decoded frame through run(); PNG goes back to the caller's decoder; a broken JPEG is a
    ValueError like PIL's."""
    import asyncio
    import types

    from inference_arena_amd.processing.transforms import load_image_from_bytes
    from inference_arena_amd.server.batching import AsyncBatcher

    C = native()
    runner = types.SimpleNamespace(ex=C.EchoInstance(2, 8, 4, 200))
    b = AsyncBatcher([runner], max_batch=8, max_queue_delay_us=500)
    if not jpeg_device:  # host reconstruction mode of the ingest
        b._ingest = C.JpegIngest(b._b, {"threads": 2, "jpeg_device": False})
    rng = np.random.default_rng(4)
    frames = [(rng.random((30 + 5 * i, 41 + 3 * i, 3)) * 255).astype(np.uint8) for i in range(6)]
    uploads = [_enc(f, quality=85, subsampling=i % 3) for i, f in enumerate(frames)]
    png = io.BytesIO()
    Image.fromarray(frames[0]).save(png, "PNG")
    calls = []

    async def decode(data):
        calls.append(len(data))
        return load_image_from_bytes(data)

    async def go():
        a = await asyncio.gather(*(b.run_jpeg(u, decode) for u in uploads))
        r = await asyncio.gather(*(b.run(_pil(u)) for u in uploads))
        p = await b.run_jpeg(png.getvalue(), decode)
        with pytest.raises(ValueError):
            await b.run_jpeg(uploads[0][: len(uploads[0]) // 2], decode)
        return a, r, p

    try:
        a, r, p = asyncio.run(go())
    finally:
        b.close()
    for x, y in zip(a, r):
        np.testing.assert_array_equal(x["det"], y["det"])
        np.testing.assert_array_equal(x["topk_idx"], y["topk_idx"])
    assert len({x["det_count"] for x in a}) > 1
    assert calls == [len(png.getvalue())] and p["det_count"] >= 1
    st = b.ingest_stats() if jpeg_device else None
    if st is not None:
        assert st["native"] == 6 and st["fallback"] == 1 and st["errors"] == 1


def _oversubscribe(data: bytes, pattern: int) -> bytes:
    """Rewrite the first DHT table's code-length counts so that too many short codes exist (bits[1] = 3, or
    bits[1] = 2 and bits[2] = 1) while the symbol total stays the same: the segment still parses."""
    d = bytearray(data)
    p = d.find(b"\xff\xc4")
    assert p > 0
    t = p + 5  # marker, length, Tc/Th
    total = sum(d[t:t + 16])
    d[t:t + 16] = bytes(16)
    if pattern == 0:
        d[t] = 3
    else:
        d[t], d[t + 1] = 2, 1
    d[t + 15] = total - 3
    return bytes(d)


@pytest.mark.parametrize("pattern", [0, 1])
def test_oversubscribed_huffman_table_is_corrupt(pattern):
    """An over-subscribed DHT must be rejected before any lookahead table is filled (the code index
    would run past the 2048-entry fast tables; libjpeg's jdhuff.c rejects code >= 1 << length)."""
    C = native()
    bad = _oversubscribe(_enc(_scene(48, 64), quality=90), pattern)
    st, err, rgb = C.jpeg_decode_host(bad)
    assert st == "corrupt" and rgb is None and "DHT" in err, (st, err)


def test_decoder_fuzz_under_address_sanitizer(tmp_path):
    """The host decoder (csrc/runtime/jpeg_decode.cpp) built host-only with AddressSanitizer and driven by
    csrc/tests/jpeg_fuzz.cpp: over-subscribed tables rejected, 2000 random mutations without a memory error."""
    import os
    import shutil
    import subprocess
    from pathlib import Path

    root = Path(__file__).resolve().parents[1]
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    if not (Path(hipcc).exists() or shutil.which(hipcc)):
        pytest.skip("hipcc not available")
    srcs = [root / "csrc" / "tests" / "jpeg_fuzz.cpp", root / "csrc" / "runtime" / "jpeg_decode.cpp"]
    exe = root / "build" / "jpeg_fuzz_address"
    exe.parent.mkdir(parents=True, exist_ok=True)
    newest = max(p.stat().st_mtime for p in srcs + [root / "csrc" / "runtime" / "jpeg_decode.h",
                                                   root / "csrc" / "kernels" / "jpeg_math.h"])
    if not exe.exists() or exe.stat().st_mtime < newest:
        cmd = [hipcc, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-Xarch_host", "-fsanitize=address",
               "-I" + str(root / "csrc"), *map(str, srcs), "-o", str(exe)]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-4000:]
    seed = tmp_path / "seed.jpg"
    seed.write_bytes(_enc(_scene(96, 128), quality=90, subsampling=2))
    r = subprocess.run([str(exe), str(seed), "2000"], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1"))
    report = r.stdout + r.stderr
    assert "AddressSanitizer" not in report and r.returncode == 0, report[-6000:]
    assert "jpeg_fuzz: ok" in r.stdout


def test_entropy_bench_builds_and_runs(tmp_path):
    """csrc/tests/jpeg_entropy_bench.cpp (host entropy-decode throughput of the split decoder) builds host-only,
    decodes a 4:2:0 upload and reports a stable coefficient checksum."""
    import shutil
    import subprocess
    from pathlib import Path

    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("g++ not available")
    root = Path(__file__).resolve().parents[1]
    exe = tmp_path / "jpeg_entropy_bench"
    r = subprocess.run([gxx, "-O2", "-std=c++17", "-I" + str(root / "csrc"),
                        str(root / "csrc" / "tests" / "jpeg_entropy_bench.cpp"),
                        str(root / "csrc" / "runtime" / "jpeg_decode.cpp"), "-o", str(exe)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    f = tmp_path / "a.jpg"
    f.write_bytes(_enc(_scene(96, 128), quality=90, subsampling=2))
    outs = [subprocess.run([str(exe), str(f)], capture_output=True, text=True, timeout=120) for _ in range(2)]
    for o in outs:
        assert o.returncode == 0 and "us per image" in o.stdout, o.stdout + o.stderr
    sums = [o.stdout.split("checksum")[1].strip() for o in outs]
    assert sums[0] == sums[1] and sums[0] != "0" * 16
