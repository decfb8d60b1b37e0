"""Serving topologies on the MI355X: every arm's GPU backend behind its real front-end."""
from __future__ import annotations

import asyncio

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def repo(tmp_path_factory):
    from inference_arena_amd.repository import store

    root = tmp_path_factory.mktemp("model_repository")
    store.build_repository(root, seed=0)
    return root


@pytest.fixture(scope="module")
def gpu_server(repo, device):
    from inference_arena_amd.server.modelserver_core import ModelServer

    ms = ModelServer(repo, device="gpu")
    assert not ms.failed, ms.failed
    yield ms
    ms.close()


def test_model_server_tensor_models(gpu_server):
    from inference_arena_amd.data.curator import workload_images
    from inference_arena_amd.processing import MobileNetPreprocessor, YOLOPreprocessor

    imgs = workload_images(3)
    xm = MobileNetPreprocessor().preprocess_batch(imgs)
    xy = YOLOPreprocessor()(imgs[0]).tensor

    async def go():
        a = await gpu_server.infer("mobilenetv2", {"input": xm})
        b = await gpu_server.infer("yolov5n", {"images": xy})
        return a["output"], b["output0"]

    ym, yy = asyncio.run(go())
    assert ym.shape == (3, 1000) and yy.shape == (1, 84, 8400)
    from inference_arena_amd.repository.store import load_module

    # the model server runs the fp32 programs: the fp32 torch modules of the repository at the fp32
    # tolerances of tests/test_fp32_gpu.py::test_fp32_tensor_models_match_torch
    with torch.no_grad():
        mref = load_module(gpu_server.entries["mobilenetv2"].model_file())
        ref = mref(torch.from_numpy(xm)).float().numpy()
        yref = load_module(gpu_server.entries["yolov5n"].model_file())
        ry = yref(torch.from_numpy(xy)).float().numpy()
    np.testing.assert_allclose(ym, ref, rtol=1e-3, atol=1e-3 * np.abs(ref).max())
    np.testing.assert_allclose(yy, ry, rtol=1e-3, atol=2e-3)
    st = gpu_server.models["mobilenetv2"].batcher.stats()
    assert st["requests"] >= 3


def test_model_server_pipeline_matches_fused(gpu_server):
    from inference_arena_amd.data.curator import workload_images
    from inference_arena_amd.data.synthetic import encode_png
    from inference_arena_amd.engine.pipeline import GpuPipeline
    from inference_arena_amd.models.zoo import default_models

    imgs = workload_images(4)

    async def go():
        outs = []
        for im in imgs:
            a = np.empty(1, dtype=object)
            a[0] = encode_png(im)
            outs.append(await gpu_server.infer("arena_pipeline", {"IMAGE_BYTES": a}))
        return outs

    outs = asyncio.run(go())
    direct = GpuPipeline(*default_models(0), device=0, buckets=[4]).infer(imgs)
    for o, d in zip(outs, direct):
        assert o["DETECTIONS"].shape[0] == len(d) >= 1
        det_ms, cls_ms, _q, gpu_ms = (float(v) for v in o["STAGE_MS"])  # device stage times of the batch
        assert det_ms > 0 and cls_ms > 0 and det_ms + cls_ms <= gpu_ms
        # bucket 4 here vs the model server's buckets: separately tuned tilings, fp32 summation order
        np.testing.assert_allclose(o["DETECTIONS"][:, :4], d.boxes, rtol=2e-5, atol=5e-3)
        np.testing.assert_array_equal(o["CLASS_IDS"], d.topk_idx)


def test_monolithic_gpu_concurrent_requests():
    import httpx

    from inference_arena_amd.data.curator import workload_images
    from inference_arena_amd.data.synthetic import encode_jpeg
    from inference_arena_amd.models.zoo import default_models
    from inference_arena_amd.server.backends import GpuBatchedBackend
    from inference_arena_amd.server.monolithic import create_app
    from inference_arena_amd.server.multipart import encode_multipart
    from inference_arena_amd.utils.settings import Settings

    be = GpuBatchedBackend(*default_models(0), device=0, max_batch=8, max_queue_delay_us=2000)
    app = create_app(Settings(LOG_LEVEL="WARNING"), be)
    imgs = workload_images(16)
    bodies = [encode_multipart("file", encode_jpeg(im)) for im in imgs]

    async def go():
        async with app.router.lifespan_context(app):
            tr = httpx.ASGITransport(app=app)
            async with httpx.AsyncClient(transport=tr, base_url="http://t") as c:
                rs = await asyncio.gather(*(c.post("/predict", content=b, headers={"content-type": t})
                                            for b, t in bodies))
        return rs

    rs = asyncio.run(go())
    assert all(r.status_code == 200 for r in rs), [r.text for r in rs if r.status_code != 200][:1]
    n = [len(r.json()["detections"]) for r in rs]
    assert np.mean(n) > 2.5
    assert max(r.json()["timing"]["batch_size"] for r in rs) > 1  # requests were batched together


def test_classification_service_gpu_batch():
    from inference_arena_amd.data.curator import workload_images
    from inference_arena_amd.models.zoo import default_models
    from inference_arena_amd.proto import inference_api as pb
    from inference_arena_amd.server.classification_service import ClassificationServicer
    from inference_arena_amd.server.crop_codec import encode_crop
    from inference_arena_amd.server.service_backends import GpuClassifierBackend

    be = GpuClassifierBackend(default_models(0)[1], device=0, max_batch=16, max_queue_delay_us=1000)
    sv = ClassificationServicer(be, [f"c{i}" for i in range(1000)])
    im = workload_images(1)[0]
    crops = [im[10 * i: 10 * i + 90, 20 * i: 20 * i + 120] for i in range(6)]
    req = pb.BatchClassificationRequest(requests=[pb.ClassificationRequest(request_id=str(i),
                                                                           image_crop=encode_crop(c, "raw"))
                                                  for i, c in enumerate(crops)])
    resp = asyncio.run(sv.ClassifyBatch(req))
    direct = [be.runners[0].infer([c])[0] for c in crops]
    for r, (idx, _, prob) in zip(resp.responses, direct):
        assert r.error == ""
        assert r.result.class_id == int(idx[0])
        assert abs(r.result.confidence - float(prob[0])) < 1e-5
    assert be.stats()["mean_batch"] > 1
    be.close()
