#!/usr/bin/env python3
"""Engine-only driver for rocprofv3: runs ``--batches`` full batches of the curated workload through
one GpuPipeline (``--dtype``), sequentially, so a kernel trace maps one graph replay per batch onto
the program's ops (tools/analyze_trace.py)."""
from __future__ import annotations

import argparse
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="fp32")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--batches", type=int, default=20)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--inputs", default="rgb", choices=["rgb", "jpeg"],
                    help="rgb: decoded frames (host pack); jpeg: the HTTP path's device inputs (JPEG q90 uploads "
                         "entropy-decoded once into pinned buffers: coefficient H2D + GPU reconstruction per batch)")
    a = ap.parse_args(argv)
    import torch

    from inference_arena_amd.data.curator import DatasetManifest, load_manifest_images
    from inference_arena_amd.engine.pipeline import GpuPipeline
    from inference_arena_amd.models.zoo import default_models

    root = Path(__file__).resolve().parents[1]
    sfx = "" if a.dtype == "fp32" else f"_{a.dtype}"
    man = DatasetManifest.load(root / "data" / "synthetic_set" / f"manifest_w{a.seed}_n100{sfx}.json")
    images = load_manifest_images(man)
    pipe = GpuPipeline(*default_models(a.seed), device=0, buckets=[a.batch], dtype=a.dtype)
    B = a.batch
    if a.inputs == "jpeg":
        from inference_arena_amd.data.synthetic import encode_jpeg
        from inference_arena_amd.ops import native

        js = native().JpegSet([encode_jpeg(im, int(man.config.get("jpeg_quality", 90))) for im in images])

        def run(i):
            return pipe.ex.collect(pipe.ex.submit_jpeg_set(js, [(i * B + k) % len(images) for k in range(B)]))
    else:
        def run(i):
            return pipe.ex.run([images[(i * B + k) % len(images)] for k in range(B)])
    for i in range(3):
        run(i)
    torch.cuda.synchronize()
    t = time.perf_counter()
    gpu = []
    for i in range(a.batches):
        r = run(i)
        gpu.append(r["gpu_ms"])
    dt = time.perf_counter() - t
    gpu.sort()
    if a.inputs == "jpeg":
        # the coefficient bytes one batch DMAs from pinned memory, and the time of one copy of that size
        # (pinned host -> device, timed by events) - the H2D share of the split decoder per batch
        nbytes = int(sum(js.coef_bytes(k % len(images)) for k in range(B)))
        h = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
        d = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(3):
            d.copy_(h, non_blocking=True)
        e0.record()
        for _ in range(10):
            d.copy_(h, non_blocking=True)
        e1.record()
        torch.cuda.synchronize()
        print(f"jpeg coefficients per batch of {B}: {nbytes / 1e6:.2f} MB, pinned H2D {e0.elapsed_time(e1) / 10 * 1e3:.1f} us",
              flush=True)
        del js
    print(f"{a.dtype} ({a.inputs}): {a.batches} sequential batches of {B}: {dt / a.batches * 1e3:.3f} ms/batch wall, "
          f"gpu_ms p50 {gpu[len(gpu) // 2]:.3f}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
