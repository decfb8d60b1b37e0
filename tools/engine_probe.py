#!/usr/bin/env python3
"""Engine-only throughput probe: the fp32 pipeline fed pre-decoded workload images through submit/collect
(bench.py engine_throughput), to separate device-bound from host-staging-bound rates.  Knobs come from the
environment (ARENA_SLOTS, ARENA_CONCURRENCY, ARENA_DEBUG_SKIP_PACK, ...)."""
from __future__ import annotations

import argparse
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--batches", type=int, default=150)
    ap.add_argument("--dtype", default="fp32")
    ap.add_argument("--inputs", default="rgb", choices=["rgb", "jpeg"],
                    help="rgb: decoded frames packed on the host (engine_rgb_req_s); jpeg: the workload encoded as "
                         "JPEG q90 and entropy-decoded once into pinned buffers, coefficient H2D + GPU "
                         "reconstruction per batch (bench.py engine_req_s)")
    a = ap.parse_args(argv)
    import torch

    import bench
    from inference_arena_amd.engine.pipeline import GpuPipeline
    from inference_arena_amd.models.zoo import default_models
    from inference_arena_amd.parallel.dist import DistInfo

    torch.cuda.set_device(0)
    yolo, mnet = default_models(0)
    pipe = GpuPipeline(yolo, mnet, device=0, buckets=sorted({1, a.batch}), dtype=a.dtype)
    info = DistInfo(rank=0, world=1, local_rank=0, backend="none")
    images, man = bench.load_workload(pipe, info, 100, 0, a.dtype)
    jset = None
    if a.inputs == "jpeg":
        from inference_arena_amd.data.synthetic import encode_jpeg
        from inference_arena_amd.ops import native

        q = int(man.config.get("jpeg_quality", 90))
        jset = native().JpegSet([encode_jpeg(im, q) for im in images], pinned=True)
    bench.engine_throughput(pipe.ex, images, a.batch, 10, jset)
    t = time.perf_counter()
    r = bench.engine_throughput(pipe.ex, images, a.batch, a.batches, jset)
    knobs = {k: v for k, v in os.environ.items() if k.startswith("ARENA_")}
    print(f"engine {r:.0f} req/s ({a.inputs}, {a.batches} batches of {a.batch}, {time.perf_counter() - t:.1f}s) {knobs}", flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
