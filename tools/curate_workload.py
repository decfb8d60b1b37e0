#!/usr/bin/env python3
"""Curate the synthetic workload with the GPU pipeline of a given precision (reference protocol:
src/shared/data/curator.py:480-678 — images with 3-5 detections at conf 0.5 / IoU 0.45, balanced
25/50/25 sampling with seed 42) and write its manifest.

    python tools/curate_workload.py --dtype fp32 --out data/synthetic_set/manifest_w0_n100.json
"""
from __future__ import annotations

import argparse
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="fp32")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--n", type=int, default=100)
    ap.add_argument("--out", required=True)
    ap.add_argument("--jpeg-quality", type=int, default=90,
                    help="count detections on the JPEG round trip the load generator sends (0: raw pixels)")
    a = ap.parse_args(argv)
    from inference_arena_amd.data.curator import CurationConfig, curate
    from inference_arena_amd.engine.pipeline import GpuPipeline
    from inference_arena_amd.models.zoo import default_models

    from inference_arena_amd.data.synthetic import encode_jpeg
    from inference_arena_amd.processing.transforms import load_image_from_bytes

    pipe = GpuPipeline(*default_models(a.seed), device=0, buckets=[32], dtype=a.dtype)
    q = a.jpeg_quality

    def count(imgs):
        # the reference curates the JPEG files its load test sends (src/shared/data/curator.py:480-599):
        # count on the decoded upload, not on the pre-encoding pixels
        if q > 0:
            imgs = [load_image_from_bytes(encode_jpeg(im, q)) for im in imgs]
        return [len(r) for r in pipe.infer(imgs)]

    t = time.time()
    _, man = curate(count, CurationConfig(target_count=a.n), log=lambda *x: print(*x, file=sys.stderr))
    man.config["weight_seed"] = a.seed
    man.config["dtype"] = a.dtype
    man.config["jpeg_quality"] = q
    man.save(Path(a.out))
    print(f"curated {len(man.images)} images in {time.time() - t:.1f}s: {man.statistics} -> {a.out}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
