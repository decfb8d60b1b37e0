"""Staggered launch of concurrent batches (csrc/runtime/executor.cpp capture / launch_graph, ARENA_STAGGER).

A bucket's graph is captured in parts; a full batch launched while two others are in flight waits, on the device,
for the previously launched batch to finish each gated part.  The kernels and their order within a batch are
unchanged, so every answer must be bit-identical to the unsplit program's, whatever the split points and however
many batches overlap (profiles/r6_stagger/README.md)."""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def workload():
    from inference_arena_amd.data.curator import workload_images
    from inference_arena_amd.data.synthetic import encode_jpeg
    from inference_arena_amd.models.zoo import default_models
    from inference_arena_amd.ops import native

    jpegs = [encode_jpeg(im, 90) for im in workload_images(64)]
    return default_models(0), native().JpegSet(jpegs, pinned=True)


def _pipelined(pipe, js, batches: int):
    """``batches`` full batches of 32, submitted ahead up to every staging slot, collected in order."""
    from inference_arena_amd.engine.pipeline import split_results

    depth = pipe.ex.num_slots()
    q, out = [], []
    for k in range(batches):
        q.append(pipe.ex.submit_jpeg_set(js, [(32 * k + i) % len(js) for i in range(32)]))
        if len(q) == depth:
            out.append(split_results(pipe.ex.collect(q.pop(0)), 32))
    while q:
        out.append(split_results(pipe.ex.collect(q.pop(0)), 32))
    return out


@pytest.mark.parametrize("stagger", ["0.25", "0.2,0.45", "0.15,0.35,0.6"])
def test_staggered_batches_match_the_unsplit_program(workload, stagger, monkeypatch):
    from inference_arena_amd.engine.pipeline import GpuPipeline

    models, js = workload
    monkeypatch.setenv("ARENA_STAGGER", "0")
    base = GpuPipeline(*models, device=0, buckets=[32], dtype="fp32")
    want = _pipelined(base, js, 2)
    del base
    monkeypatch.setenv("ARENA_STAGGER", stagger)
    pipe = GpuPipeline(*models, device=0, buckets=[32], dtype="fp32")
    got = _pipelined(pipe, js, 10)  # 10 batches over 4 slots: the gated waits are exercised
    for k, batch in enumerate(got):
        for x, y in zip(batch, want[k % 2]):
            np.testing.assert_array_equal(x.boxes, y.boxes)
            np.testing.assert_array_equal(x.topk_idx, y.topk_idx)
            np.testing.assert_array_equal(x.topk_logit, y.topk_logit)
