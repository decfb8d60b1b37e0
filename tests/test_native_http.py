"""Native HTTP front end (csrc/runtime/http_front.h) end to end on CPU: real sockets, the spawned PIL
decode processes (native-mode decode pool) and the native dynamic batcher over the host-only
EchoInstance.  Pins the /predict wire contract of server/monolithic.py (reference
architectures/monolithic/app/main.py): JSON schema, label names, error codes, keep-alive, chunked
bodies and concurrent clients."""
from __future__ import annotations

import http.client
import io
import json
import threading

import numpy as np
import pytest
from PIL import Image

from inference_arena_amd.labels import load_labels
from inference_arena_amd.ops import native
from inference_arena_amd.server.native_front import NativeFrontEnd


def _jpeg(h, w, first):
    arr = np.full((h, w, 3), 128, np.uint8)
    arr[:8, :8] = first  # the decoded first pixel picks the echo instance's detection count
    b = io.BytesIO()
    Image.fromarray(arr).save(b, format="PNG")  # lossless: the first byte survives the round trip
    return b.getvalue()


def _multipart(data: bytes, field="file"):
    bnd = "arenaboundary123"
    body = (f"--{bnd}\r\nContent-Disposition: form-data; name=\"{field}\"; filename=\"x.png\"\r\n"
            f"Content-Type: image/png\r\n\r\n").encode() + data + f"\r\n--{bnd}--\r\n".encode()
    return body, f"multipart/form-data; boundary={bnd}"


@pytest.fixture(scope="module")
def server():
    C = native()
    batcher = C.DynamicBatcher([C.EchoInstance(2, 8, 4, 1000)], {"max_batch": 8, "max_queue_delay_us": 200})
    labels = load_labels(None)
    fe = NativeFrontEnd(batcher, labels, port=0, host="127.0.0.1", io_threads=2, decode_procs=2, slots=16)
    yield fe, labels
    fe.close()
    batcher.shutdown()


def _post(port, body, ctype, conn=None, headers=None):
    c = conn or http.client.HTTPConnection("127.0.0.1", port, timeout=30)
    c.request("POST", "/predict", body=body, headers={"Content-Type": ctype, **(headers or {})})
    r = c.getresponse()
    data = r.read()
    return r.status, data, c


def test_predict_schema_and_labels(server):
    fe, labels = server
    body, ct = _multipart(_jpeg(48, 64, 2))
    st, data, c = _post(fe.port, body, ct)
    assert st == 200
    d = json.loads(data)
    assert set(d) == {"request_id", "detections", "timing"} and len(d["request_id"]) == 36
    assert len(d["detections"]) == 3  # 1 + first_byte % max_det
    for k, det in enumerate(d["detections"]):
        box = det["detection"]
        assert (box["x1"], box["y1"], box["x2"], box["y2"]) == (k, k, 64 - k, 48 - k)
        assert box["class_id"] == k and abs(box["confidence"] - (0.9 - 0.1 * k)) < 1e-6
        cls = det["classification"]
        assert cls["class_id"] == 10 * k and cls["class_name"] == labels[10 * k] and cls["confidence"] == 5.0
    for key in ("queue_ms", "gpu_ms", "batch_size", "detection_ms", "classification_ms", "inference_ms",
                "decode_ms", "total_ms"):
        assert key in d["timing"]
    # keep-alive: a second request on the same connection
    st2, data2, _ = _post(fe.port, body, ct, conn=c)
    assert st2 == 200 and json.loads(data2)["request_id"] != d["request_id"]
    c.close()


def test_raw_body_chunked_and_errors(server):
    fe, _ = server
    img = _jpeg(32, 32, 0)
    st, data, c = _post(fe.port, img, "image/png")
    assert st == 200 and len(json.loads(data)["detections"]) == 1
    c.close()
    # chunked transfer encoding
    c = http.client.HTTPConnection("127.0.0.1", fe.port, timeout=30)
    c.request("POST", "/predict", body=iter([img[:100], img[100:]]), headers={"Content-Type": "image/png"},
              encode_chunked=True)
    r = c.getresponse()
    assert r.status == 200 and len(json.loads(r.read())["detections"]) == 1
    c.close()
    body, ct = _multipart(img, field="other")
    st, data, c = _post(fe.port, body, ct)
    assert st == 422 and "file" in json.loads(data)["detail"]
    c.close()
    st, data, c = _post(fe.port, b"not an image", "image/jpeg")
    assert st == 500 and "Failed to decode image" in json.loads(data)["detail"]
    c.close()
    st, data, c = _post(fe.port, b"", "image/jpeg")
    assert st == 422
    c.close()
    c = http.client.HTTPConnection("127.0.0.1", fe.port, timeout=30)
    c.request("GET", "/nope")
    assert c.getresponse().status == 404
    c.close()


def test_health_metrics_and_concurrency(server):
    fe, _ = server
    c = http.client.HTTPConnection("127.0.0.1", fe.port, timeout=30)
    c.request("GET", "/health")
    r = c.getresponse()
    assert r.status == 200 and json.loads(r.read()) == {"status": "healthy", "models_loaded": True}
    errors, n_ok = [], []

    def worker(i):
        try:
            conn = http.client.HTTPConnection("127.0.0.1", fe.port, timeout=30)
            for j in range(6):
                body, ct = _multipart(_jpeg(24 + i, 40, (i + j) % 4))
                st, data, conn = _post(fe.port, body, ct, conn=conn)
                assert st == 200, data
                assert len(json.loads(data)["detections"]) == 1 + (i + j) % 4
                n_ok.append(1)
            conn.close()
        except Exception as e:  # noqa: BLE001
            errors.append(e)
    ts = [threading.Thread(target=worker, args=(i,)) for i in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors and len(n_ok) == 48
    # one failed request of this test's own (the module's other tests may run in another xdist worker)
    st, data, c2 = _post(fe.port, b"not an image", "image/jpeg")
    assert st == 500
    c2.close()
    s = fe.stats()
    assert s["ok"] >= 48 and s["errors"] >= 1
    import time

    # the metrics text refreshes once a second; poll (a loaded CI host can be late)
    c.close()
    deadline = time.monotonic() + 10.0
    while True:
        time.sleep(0.3)
        c = http.client.HTTPConnection("127.0.0.1", fe.port, timeout=30)
        c.request("GET", "/metrics")
        r = c.getresponse()
        text = r.read().decode()
        ok = r.status == 200 and 'arena_requests_total{arch="monolithic",status="ok"}' in text
        if ok or time.monotonic() > deadline:
            break
        c.close()
    assert ok, text[:400]
    fe.set_healthy(False)
    c.request("GET", "/health")
    r = c.getresponse()
    assert r.status == 503 and json.loads(r.read())["status"] == "unhealthy"
    fe.set_healthy(True)
    c.close()


@pytest.fixture(scope="module")
def tight_server():
    """A front end with a 1 MB body limit and short timeouts (the hardening paths)."""
    C = native()
    batcher = C.DynamicBatcher([C.EchoInstance(2, 8, 4)], {"max_batch": 8, "max_queue_delay_us": 200})
    fe = NativeFrontEnd(batcher, load_labels(None), port=0, host="127.0.0.1", io_threads=2, decode_procs=1,
                        slots=8, max_body=1 << 20, idle_timeout_ms=1500, read_timeout_ms=1500)
    yield fe
    fe.close()
    batcher.shutdown()


def _raw(port, data: bytes, read_timeout=10.0) -> bytes:
    import socket

    s = socket.create_connection(("127.0.0.1", port), timeout=read_timeout)
    try:
        s.sendall(data)
        out = b""
        while True:
            try:
                k = s.recv(65536)
            except (ConnectionResetError, socket.timeout):
                break
            if not k:
                break
            out += k
            if b"\r\n\r\n" in out and b"Connection: close" in out:
                break
        return out
    finally:
        s.close()


def test_chunked_overflow_and_saturated_size_rejected(tight_server):
    """A chunk size that saturates strtoll (or simply exceeds the body limit) is a 413, not an endless wait
    (the signed sum overflowed and bypassed max_body)."""
    fe = tight_server
    head = b"POST /predict HTTP/1.1\r\nHost: x\r\nTransfer-Encoding: chunked\r\nContent-Type: image/png\r\n\r\n"
    r = _raw(fe.port, head + b"7fffffffffffffffffff\r\nabc")
    assert r.startswith(b"HTTP/1.1 413"), r[:80]
    r = _raw(fe.port, head + b"200000\r\n" + b"x" * 100)  # 2 MB chunk > 1 MB limit, announced up front
    assert r.startswith(b"HTTP/1.1 413"), r[:80]
    r = _raw(fe.port, head + b"zz\r\n")
    assert r.startswith(b"HTTP/1.1 400"), r[:80]


def test_pipelined_flood_does_not_grow_unbounded(tight_server):
    """A client that keeps sending while its request is in flight is read up to one maximal request, then
    paused; its first request is still answered and the server keeps serving others."""
    import socket

    fe = tight_server
    body, ct = _multipart(_jpeg(16, 16, 1))
    req = (f"POST /predict HTTP/1.1\r\nHost: x\r\nContent-Type: {ct}\r\nContent-Length: {len(body)}\r\n\r\n"
           ).encode() + body
    s = socket.create_connection(("127.0.0.1", fe.port), timeout=10)
    sent = 0
    junk = b"GET /health HTTP/1.1\r\nHost: x\r\n\r\n" * 2000
    try:
        s.sendall(req)
        s.setblocking(False)
        for _ in range(400):  # ~27 MB offered: far beyond the 1 MB + 64 KB input cap
            try:
                sent += s.send(junk)
            except BlockingIOError:
                break
        assert sent < 8 << 20  # the kernel buffers filled: the server stopped reading
    finally:
        s.close()
    st, _, c = _post(fe.port, body, ct)  # still serving
    assert st == 200
    c.close()


def test_idle_and_trickling_connections_time_out(tight_server):
    import socket
    import time

    fe = tight_server
    before = fe.stats()["timeouts"]
    idle = socket.create_connection(("127.0.0.1", fe.port), timeout=10)
    trickle = socket.create_connection(("127.0.0.1", fe.port), timeout=10)
    trickle.sendall(b"POST /predict HTTP/1.1\r\nHost: x\r\n")  # headers never finish
    t0 = time.time()
    for s in (idle, trickle):
        assert s.recv(1) == b""  # closed by the server
    assert 1.0 < time.time() - t0 < 8.0
    assert fe.stats()["timeouts"] >= before + 2
    idle.close()
    trickle.close()


def _http_request(body: bytes, ctype: str) -> bytes:
    return (f"POST /predict HTTP/1.1\r\nHost: 127.0.0.1\r\nContent-Type: {ctype}\r\nContent-Length: {len(body)}\r\n"
            f"\r\n").encode() + body


def test_native_load_generator_closed_loop(server):
    """The native closed-loop client (csrc/runtime/http_loadgen.cpp, bench.py's HTTP path): every response
    is counted once, with its status and its detection count parsed from the JSON."""
    fe, _ = server
    reqs = []
    for first in (1, 2, 3, 4):
        body, ct = _multipart(_jpeg(24, 32, first))
        reqs.append(_http_request(body, ct))
    lg = native().HttpLoadGen({"host": "127.0.0.1", "port": fe.port, "users": 8, "threads": 2}, reqs)
    lg.start()
    assert lg.wait_completed(400, 60)
    lg.stop(30)
    r = lg.records(0, -1)
    n = len(r["latency"])
    assert n >= 400 and lg.completed() == n
    assert (r["status"] == 200).all()
    assert set(r["dets"].tolist()) <= {2, 3, 4, 1} and (r["latency"] > 0).all()
    assert (np.diff(r["t_done"]) >= 0).all()  # completion order


def test_stage_timing_and_stage_histograms(server):
    """detection_ms / classification_ms are the device stage times of the request's batch (never the old
    constants): positive, and together no more than gpu_ms; /metrics exports a histogram per stage."""
    import urllib.request

    fe, _ = server
    body, ct = _multipart(_jpeg(40, 40, 3))
    st, data, c = _post(fe.port, body, ct)
    c.close()
    t = json.loads(data)["timing"]
    assert st == 200 and t["detection_ms"] > 0 and t["classification_ms"] > 0
    assert t["detection_ms"] + t["classification_ms"] <= t["gpu_ms"] + 1e-6
    stages = fe.stats()["stages"]
    assert set(stages) == {"decode", "queue", "gpu", "detection", "classification", "total"}
    assert all(sum(h) >= 1 for h, _ in stages.values())
    fe.fe.set_metrics_text(__import__("prometheus_client").generate_latest(fe.registry).decode())
    with urllib.request.urlopen(f"http://127.0.0.1:{fe.port}/metrics", timeout=10) as r:
        text = r.read().decode()
    for stage in ("decode", "queue", "gpu", "detection", "classification", "total"):
        assert f'arena_request_latency_seconds_count{{arch="monolithic",stage="{stage}"}}' in text


_FRONT_SRCS = ["csrc/tests/front_stress.cpp", "csrc/runtime/http_front.cpp", "csrc/runtime/kserve.cpp", "csrc/runtime/batcher.cpp",
               "csrc/runtime/trace.cpp", "csrc/runtime/jpeg_decode.cpp"]


@pytest.mark.parametrize("sanitizer", ["thread", "address"])
def test_front_end_stress_under_sanitizer(sanitizer):
    """The native HTTP front end (I/O threads, collector, batcher threads, handler-mode owners) under TSAN /
    ASAN: keep-alive and pipelined clients with checked answers, half-close, oversized headers, malformed
    requests, decoder errors, oversize results on the worker pipe, dropped connections, drain() and stop()
    under load (csrc/tests/front_stress.cpp)."""
    import os
    import shutil
    import subprocess
    from pathlib import Path

    root = Path(__file__).resolve().parents[1]
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    if not (Path(hipcc).exists() or shutil.which(hipcc)):
        pytest.skip("hipcc not available")
    srcs = [root / s for s in _FRONT_SRCS]
    out = root / "build" / f"front_stress_{sanitizer}"
    out.parent.mkdir(parents=True, exist_ok=True)
    newest = max(p.stat().st_mtime for p in srcs + list((root / "csrc" / "runtime").glob("*.h")))
    if not out.exists() or out.stat().st_mtime < newest:
        cmd = [hipcc, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-Xarch_host", f"-fsanitize={sanitizer}",
               "-I" + str(root / "csrc"), *map(str, srcs), "-ldl", "-o", str(out)]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, r.stderr[-4000:]
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1:second_deadlock_stack=1",
               ASAN_OPTIONS="detect_leaks=1:halt_on_error=1")
    r = subprocess.run([str(out)], capture_output=True, text=True, timeout=600, env=env)
    report = r.stdout + r.stderr
    assert "ThreadSanitizer" not in report and "AddressSanitizer" not in report, report[-6000:]
    assert r.returncode == 0, report[-6000:]
    assert "front_stress: ok" in r.stdout


def test_tiny_chunks_beyond_the_input_cap_get_413():
    """A chunked upload whose wire size passes max_body + 64 KiB while its decoded body stays under max_body
    is answered 413 (it used to sit paused until the read timeout closed it without a status)."""
    import socket

    C = native()
    batcher = C.DynamicBatcher([C.EchoInstance(2, 8, 4, 0)], {"max_batch": 8, "max_queue_delay_us": 200})
    fe = NativeFrontEnd(batcher, load_labels(None), port=0, host="127.0.0.1", io_threads=1, decode_procs=1, slots=4,
                        max_body=100_000)
    try:
        s = socket.create_connection(("127.0.0.1", fe.port), timeout=20)
        s.sendall(b"POST /predict HTTP/1.1\r\nHost: x\r\nTransfer-Encoding: chunked\r\nContent-Type: image/jpeg\r\n\r\n")
        chunk = b"1\r\nX\r\n" * 4096  # 6 wire bytes per body byte
        resp = b""
        try:
            for _ in range(60):  # ~1.4 MB on the wire, 240 KB decoded... the server answers well before that
                s.sendall(chunk)
        except (BrokenPipeError, ConnectionResetError):
            pass
        s.settimeout(20)
        try:
            while b"\r\n\r\n" not in resp:
                d = s.recv(65536)
                if not d:
                    break
                resp += d
        except ConnectionResetError:
            pass
        assert resp.startswith(b"HTTP/1.1 413"), resp[:200]
        s.close()
    finally:
        fe.close()
        batcher.shutdown()


@pytest.mark.parametrize("jpeg_device", [True, False])
def test_split_decoder_answers_like_the_pil_pool(jpeg_device):
    """JPEG uploads through the native split decoder (coefficients handed to the instance, or reconstructed on
    the host threads) answer exactly like the PIL decode processes: the echo instance's detections depend on the
    decoded first pixel, which must be bit-identical."""
    C = native()
    rng = np.random.default_rng(11)
    uploads = []
    for i in range(8):
        arr = (rng.random((40 + 8 * i, 56 + 4 * i, 3)) * 255).astype(np.uint8)
        b = io.BytesIO()
        Image.fromarray(arr).save(b, format="JPEG", quality=90, subsampling=i % 3)
        uploads.append(b.getvalue())
    answers = {}
    for threads in (3, 0):
        batcher = C.DynamicBatcher([C.EchoInstance(2, 8, 4, 200)], {"max_batch": 8, "max_queue_delay_us": 200})
        fe = NativeFrontEnd(batcher, load_labels(None), port=0, host="127.0.0.1", io_threads=2, decode_procs=1,
                            slots=16, decode_threads=threads, jpeg_device=jpeg_device)
        try:
            out = []
            for u in uploads:
                body, ct = _multipart(u)
                st, data, c = _post(fe.port, body, ct)
                c.close()
                assert st == 200
                out.append([(d["detection"], d["classification"]) for d in json.loads(data)["detections"]])
            answers[threads] = out
            s = fe.stats()
            assert (s["native_decoded"], s["fallback_decoded"]) == ((8, 0) if threads else (0, 8))
            if threads:  # request bodies come back from the decode threads to the body pool (string_pool.h)
                assert s["bodies_recycled"] >= 4, s
        finally:
            fe.close()
            batcher.shutdown()
    assert answers[3] == answers[0]
    assert len({len(a) for a in answers[3]}) > 1  # the first pixels differ, so the checks are not vacuous


def test_split_decoder_stages_oversize_frames_as_rgb():
    """a JPEG whose coefficients + sample planes + RGB frame exceed one batch's staging pool (about
    > 15 MP at 4:2:0 with the executor's default pool) used to get a 413 from the split decoder although the PIL
    path serves it as RGB.  Here the instance's staging pool is 3 x the frame's RGB bytes (as the default pool is
    3 x 640 x 640 x 3 per image): the frame is reconstructed on the host and staged as RGB, with the same answer."""
    C = native()
    h, w = 96, 128
    arr = (np.random.default_rng(5).random((h, w, 3)) * 255).astype(np.uint8)
    b = io.BytesIO()
    Image.fromarray(arr).save(b, format="JPEG", quality=90, subsampling=0)  # 4:4:4: coefficients 6 B / px
    upload = b.getvalue()
    answers = []
    for cap in (0, h * w * 3 * 3):
        batcher = C.DynamicBatcher([C.EchoInstance(2, 8, 4, 200, cap)], {"max_batch": 8, "max_queue_delay_us": 200})
        fe = NativeFrontEnd(batcher, load_labels(None), port=0, host="127.0.0.1", io_threads=2, decode_procs=1,
                            slots=16, decode_threads=2, jpeg_device=True)
        try:
            body, ct = _multipart(upload)
            st, data, c = _post(fe.port, body, ct)
            c.close()
            assert st == 200, data
            answers.append([(d["detection"], d["classification"]) for d in json.loads(data)["detections"]])
            assert fe.stats()["native_decoded"] == 1
        finally:
            fe.close()
            batcher.shutdown()
    assert answers[0] == answers[1]


def test_kserve_codec_fuzz_under_address_sanitizer():
    """csrc/runtime/kserve.cpp built host-only with AddressSanitizer and driven by csrc/tests/kserve_fuzz.cpp:
    deeply nested headers (stack depth), binary_data_size values that wrap a 64-bit sum, negative sizes and
    shapes, DETECTIONS / CLASS_* shapes that disagree are all rejected; valid messages round-trip; 4000 random
    mutations parse without a memory error (kserve.cpp:59, :244, :409)."""
    import os
    import shutil
    import subprocess
    from pathlib import Path

    root = Path(__file__).resolve().parents[1]
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    if not (Path(hipcc).exists() or shutil.which(hipcc)):
        pytest.skip("hipcc not available")
    srcs = [root / "csrc" / "tests" / "kserve_fuzz.cpp", root / "csrc" / "runtime" / "kserve.cpp"]
    exe = root / "build" / "kserve_fuzz_address"
    exe.parent.mkdir(parents=True, exist_ok=True)
    newest = max(p.stat().st_mtime for p in srcs + list((root / "csrc" / "runtime").glob("*.h")))
    if not exe.exists() or exe.stat().st_mtime < newest:
        cmd = [hipcc, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-Xarch_host", "-fsanitize=address",
               "-I" + str(root / "csrc"), *map(str, srcs), "-o", str(exe)]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, r.stderr[-4000:]
    r = subprocess.run([str(exe), "4000"], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1"))
    report = r.stdout + r.stderr
    assert "AddressSanitizer" not in report and r.returncode == 0, report[-6000:]
    assert "kserve_fuzz: ok" in r.stdout


def _kserve_request(upload: bytes) -> tuple[bytes, int]:
    import struct

    hdr = json.dumps({"inputs": [{"name": "IMAGE_BYTES", "shape": [1], "datatype": "BYTES",
                                  "parameters": {"binary_data_size": len(upload) + 4}}],
                      "outputs": [{"name": n, "parameters": {"binary_data": True}}
                                  for n in ("DETECTIONS", "CLASS_IDS", "CLASS_LOGITS", "CLASS_PROBS", "STAGE_MS")]})
    hb = hdr.encode()
    return hb + struct.pack("<I", len(upload)) + upload, len(hb)


def test_kserve_rest_route_and_native_gateway():
    """The model server's native KServe-v2 REST endpoint (binary tensor extension: IMAGE_BYTES in, the ensemble's
    output tensors out) and the native gateway (proxy mode: /predict forwarded over keep-alive connections, the
    output tensors turned into the reference JSON) answer exactly what the monolithic /predict answers."""
    from inference_arena_amd.server.native_gateway import NativeGateway

    C = native()
    labels = load_labels(None)
    batcher = C.DynamicBatcher([C.EchoInstance(2, 8, 4, 200)], {"max_batch": 8, "max_queue_delay_us": 200})
    ms = NativeFrontEnd(batcher, labels, port=0, host="127.0.0.1", io_threads=2, decode_procs=1, slots=16,
                        decode_threads=2, jpeg_device=False, kserve_model="arena_pipeline")
    gw = NativeGateway(labels, upstream=f"127.0.0.1:{ms.port}", port=0, host="127.0.0.1", conns=4, io_threads=2)
    try:
        assert gw.wait_ready(10)
        c = http.client.HTTPConnection("127.0.0.1", ms.port, timeout=30)
        for path, code in (("/v2/health/live", 200), ("/v2/health/ready", 200), ("/v2/models/arena_pipeline", 200),
                           ("/v2/models/arena_pipeline/ready", 200), ("/v2/models/nope/ready", 404)):
            c.request("GET", path)
            r = c.getresponse()
            body = r.read()
            assert r.status == code, (path, r.status, body)
        c.request("GET", "/v2/models/arena_pipeline")
        meta = json.loads(c.getresponse().read())
        assert [t["name"] for t in meta["inputs"]] == ["IMAGE_BYTES"] and len(meta["outputs"]) == 5
        rng = np.random.default_rng(4)
        for i in range(6):
            arr = (rng.random((40 + 8 * i, 64, 3)) * 255).astype(np.uint8)
            b = io.BytesIO()
            Image.fromarray(arr).save(b, format="JPEG", quality=90)
            up = b.getvalue()
            # direct /predict on the model server front end (the monolithic contract)
            body, ct = _multipart(up)
            st, data, c2 = _post(ms.port, body, ct)
            c2.close()
            assert st == 200
            direct = json.loads(data)["detections"]
            # KServe infer, binary tensors
            req, ihcl = _kserve_request(up)
            c.request("POST", "/v2/models/arena_pipeline/infer", body=req,
                      headers={"Content-Type": "application/octet-stream",
                               "Inference-Header-Content-Length": str(ihcl)})
            r = c.getresponse()
            raw = r.read()
            assert r.status == 200, raw
            n = int(r.getheader("Inference-Header-Content-Length"))
            hdr = json.loads(raw[:n])
            outs, pos = {}, n
            for o in hdr["outputs"]:
                sz = o["parameters"]["binary_data_size"]
                dt = np.int32 if o["datatype"] == "INT32" else np.float32
                outs[o["name"]] = np.frombuffer(raw[pos:pos + sz], dtype=dt).reshape(o["shape"])
                pos += sz
            assert pos == len(raw) and outs["DETECTIONS"].shape == (len(direct), 6)
            for k, d in enumerate(direct):
                assert outs["CLASS_IDS"][k, 0] == d["classification"]["class_id"]
                assert outs["DETECTIONS"][k, 4] == pytest.approx(d["detection"]["confidence"])
            # through the native gateway
            st, data, c3 = _post(gw.port, body, ct)
            c3.close()
            assert st == 200, data
            via = json.loads(data)
            assert [(d["detection"], d["classification"]) for d in via["detections"]] == \
                [(d["detection"], d["classification"]) for d in direct]
            assert via["timing"]["total_ms"] > 0
        # protocol errors: no binary extension, unknown model
        c.request("POST", "/v2/models/arena_pipeline/infer", body=b'{"inputs":[]}',
                  headers={"Content-Type": "application/json"})
        r = c.getresponse()
        assert r.status == 400 and "binary tensor" in json.loads(r.read())["error"]
        c.request("POST", "/v2/models/yolov9/infer", body=b"{}", headers={"Content-Type": "application/json"})
        r = c.getresponse()
        assert r.status == 404 and "error" in json.loads(r.read())
        assert gw.stats()["ok"] == 6 and ms.stats()["ok"] == 18  # direct + KServe + via the gateway
        assert gw.stats()["bodies_recycled"] >= 3  # uploads return from the proxy workers to the body pool
    finally:
        gw.close()
        ms.close()
        batcher.shutdown()


def test_native_gateway_reports_a_dead_model_server():
    from inference_arena_amd.server.native_gateway import NativeGateway

    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        dead = s.getsockname()[1]
    gw = NativeGateway(load_labels(None), upstream=f"127.0.0.1:{dead}", port=0, host="127.0.0.1", conns=2)
    try:
        assert not gw.wait_ready(0.5)
        gw.fe.set_healthy(True)  # force: the proxy must answer 502, not hang
        body, ct = _multipart(_jpeg(16, 16, 1))
        st, data, c = _post(gw.port, body, ct)
        c.close()
        assert st == 502 and "model server" in json.loads(data)["detail"]
    finally:
        gw.close()
