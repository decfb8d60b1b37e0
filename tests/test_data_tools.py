"""Dataset utilities, detection counter, registry surface and proto text generation (CPU)."""
from __future__ import annotations

import io
import zipfile

import numpy as np
import pytest

from inference_arena_amd.data.curator import DetectionCounter
from inference_arena_amd.data.synthetic import encode_jpeg, synthetic_images


def _raw84(boxes_xywh, cls, conf, n=50):
    out = np.zeros((1, 84, n), np.float32)
    for i, (b, c, s) in enumerate(zip(boxes_xywh, cls, conf)):
        out[0, :4, i] = b
        out[0, 4 + c, i] = s
    return out


def test_detection_counter_formats():
    boxes = [(50, 50, 20, 20), (51, 51, 20, 20), (200, 200, 30, 30), (400, 100, 10, 10)]
    cls = [1, 1, 2, 3]
    conf = [0.9, 0.8, 0.7, 0.3]
    dc = DetectionCounter(0.5, 0.45)
    raw = _raw84(boxes, cls, conf)
    assert dc.count(raw) == 2  # overlapping pair suppressed, low score dropped
    assert dc.count(raw[0]) == 2
    v5 = np.zeros((1, 50, 85), np.float32)
    for i, (b, c, s) in enumerate(zip(boxes, cls, conf)):
        v5[0, i, :4] = b
        v5[0, i, 4] = 1.0
        v5[0, i, 5 + c] = s
    assert dc.count(v5) == 2
    post = np.array([[0, 0, 10, 10, 0.9, 1], [0, 0, 5, 5, 0.4, 2], [1, 1, 4, 4, 0.6, 0]], np.float32)
    assert dc.count(post[None]) == 2
    with pytest.raises(ValueError):
        dc.count(np.zeros((3, 3, 3, 3)))


def test_coco_utils(tmp_path):
    from inference_arena_amd.data import coco

    ok, msg = coco.is_coco_downloaded(tmp_path)
    assert not ok and "does not exist" in msg
    with pytest.raises(FileNotFoundError):
        coco.download_coco_val2017(tmp_path, url=None)
    buf = io.BytesIO()
    with zipfile.ZipFile(buf, "w") as z:
        for i, im in enumerate(synthetic_images(3, 1, hw=(40, 60))):
            z.writestr(f"val2017/{i:012d}.jpg", encode_jpeg(im))
    (tmp_path / "val2017.zip").write_bytes(buf.getvalue())
    with pytest.raises(RuntimeError, match="incomplete"):
        coco.download_coco_val2017(tmp_path, url=None)  # 3 images are not the 5000 of val2017
    d = coco.download_coco_val2017(tmp_path, url=None, expected_images=3)
    assert d.is_dir() and len(coco.get_coco_image_paths(tmp_path)) == 3
    assert (tmp_path / "val2017.zip").exists()  # a provided archive is kept
    ok, msg = coco.is_coco_downloaded(tmp_path)
    assert not ok and "3 of 5000" in msg
    imgs = list(coco.iter_coco_images(tmp_path, limit=2))
    assert len(imgs) == 2 and imgs[0][1].shape == (40, 60, 3)


def _zip_of(n: int) -> bytes:
    buf = io.BytesIO()
    with zipfile.ZipFile(buf, "w", compression=zipfile.ZIP_STORED) as z:
        for i, im in enumerate(synthetic_images(n, 2, hw=(32, 48))):
            z.writestr(f"val2017/{i:012d}.jpg", encode_jpeg(im))
    return buf.getvalue()


def test_coco_http_download_resumes_and_extracts(tmp_path):
    """The reference downloads val2017.zip over HTTP with a progress bar (coco_dataset.py:141-217).  Here against
    a local HTTP server with Range support: a partial .part is resumed (206), the archive is extracted, the
    downloaded zip removed, and a second call is a no-op."""
    import http.server
    import threading

    from inference_arena_amd.data import coco

    blob = _zip_of(4)
    seen = []

    class H(http.server.BaseHTTPRequestHandler):
        def do_GET(self):  # noqa: N802
            rng = self.headers.get("Range")
            seen.append(rng)
            start = int(rng.split("=")[1].split("-")[0]) if rng else 0
            body = blob[start:]
            self.send_response(206 if rng else 200)
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)

        def log_message(self, *a):
            pass

    srv = http.server.ThreadingHTTPServer(("127.0.0.1", 0), H)
    t = threading.Thread(target=srv.serve_forever, daemon=True)
    t.start()
    try:
        url = f"http://127.0.0.1:{srv.server_address[1]}/val2017.zip"
        (tmp_path / "val2017.zip.part").write_bytes(blob[:1000])  # an interrupted earlier run
        prog = []
        d = coco.download_coco_val2017(tmp_path, url=url, expected_images=4, progress=lambda a, b: prog.append((a, b)))
        assert seen == ["bytes=1000-"] and prog[-1] == (len(blob), len(blob))
        assert len(coco.get_coco_image_paths(tmp_path)) == 4 and d == tmp_path / "val2017"
        assert not (tmp_path / "val2017.zip").exists() and not (tmp_path / "val2017.zip.part").exists()
        coco.download_coco_val2017(tmp_path, url=url, expected_images=4)  # idempotent: no request
        assert len(seen) == 1
        # a fresh directory: a plain 200 download; a console progress bar
        other = tmp_path / "b"
        sink = io.StringIO()
        coco.download_coco_val2017(other, url=url, expected_images=4,
                                   progress=coco.DownloadProgress(len(blob), stream=sink))
        assert seen[-1] is None and "100%" in sink.getvalue()
        # a server that dies mid-body leaves only the .part, and the call fails loudly
        with pytest.raises(RuntimeError):
            coco.fetch_url(url.replace(str(srv.server_address[1]), "1"), tmp_path / "x.zip", timeout=2)
    finally:
        srv.shutdown()


def test_registry_surface():
    from inference_arena_amd.engine.registry import ModelRegistry, SessionConfig, get_default_registry, \
        reset_default_registry

    r = ModelRegistry(config=SessionConfig(device=0, buckets=[1, 4]))
    assert set(r.list_available()) >= {"yolov5n", "mobilenetv2", "pipeline"}
    assert not r.is_loaded("pipeline")
    with pytest.raises(KeyError):
        r._build("resnet")
    reset_default_registry()
    assert get_default_registry() is get_default_registry()
    reset_default_registry()


def test_build_session_is_the_construction_point(monkeypatch):
    """Every server backend builds its GPU models through engine.registry.build_session (one factory for
    the registry and the three serving arms); it dispatches each model kind to its engine class."""
    import inspect

    from inference_arena_amd.engine import pipeline as P
    from inference_arena_amd.engine import registry as R
    from inference_arena_amd.server import backends, modelserver_core, service_backends

    made = []

    def fake(tag):
        def ctor(*a, **kw):
            made.append((tag, kw.get("device", kw.get("det_device")), kw.get("dtype")))
            return tag
        return ctor
    monkeypatch.setattr(P, "GpuPipeline", fake("pipeline"))
    monkeypatch.setattr(P, "GpuDetector", fake("detector"))
    monkeypatch.setattr(P, "GpuClassifier", fake("classifier"))
    monkeypatch.setattr(P, "SplitPipeline", fake("split"))
    monkeypatch.setattr(P.GpuTensorModel, "yolo", classmethod(lambda cls, m, **kw: fake("yolo")(**kw)))
    monkeypatch.setattr(P.GpuTensorModel, "mobilenet", classmethod(lambda cls, m, **kw: fake("mnet")(**kw)))
    for kind, tag in (("pipeline", "pipeline"), ("detector", "detector"), ("classifier", "classifier"),
                      ("split", "split"), ("yolov5n", "yolo"), ("mobilenetv2", "mnet")):
        assert R.build_session(kind, object(), object(), device=3, buckets=[1], dtype="fp32") == tag
    assert all(d == 3 and dt == "fp32" for _, d, dt in made)
    with pytest.raises(KeyError):
        R.build_session("resnet")
    for mod in (backends, service_backends, modelserver_core):
        src = inspect.getsource(mod)
        assert "build_session(" in src
        assert "GpuPipeline(" not in src and "GpuDetector(" not in src and "GpuClassifier(" not in src


def test_generate_proto_text(tmp_path):
    import subprocess
    import sys

    subprocess.run([sys.executable, "scripts/generate_proto.py", "--out", str(tmp_path)], check=True)
    inf = (tmp_path / "inference.proto").read_text()
    assert "rpc Classify(ClassificationRequest) returns (ClassificationResponse);" in inf
    assert "bytes image_crop = 2;" in inf
    kv = (tmp_path / "kserve_v2.proto").read_text()
    assert "map<string, InferParameter> parameters = 4;" in kv and "oneof parameter_choice" in kv
    mc = (tmp_path / "model_config.proto").read_text()
    assert "repeated ModelInstanceGroup instance_group = 7;" in mc


def test_default_labels_are_the_imagenet_table():
    """The reference ships the 1000 ImageNet names and refuses to start without exactly 1000
    (reference architectures/monolithic/app/inference.py:96-125): same default here."""
    from inference_arena_amd.labels import DEFAULT_LABELS, load_labels

    labels = load_labels()
    assert len(labels) == 1000 and DEFAULT_LABELS.exists()
    assert labels[0] == "tench" and labels[1] == "goldfish" and labels[999] == "toilet tissue"
    assert len(set(labels)) > 990
