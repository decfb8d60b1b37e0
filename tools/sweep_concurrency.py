#!/usr/bin/env python3
"""Engine-only throughput vs executor concurrency: staging slots (ARENA_SLOTS) x concurrent compute
streams (ARENA_CONCURRENCY).  Each configuration builds a fresh GpuPipeline (the executor reads both
variables at construction) and runs bench.engine_throughput on the curated workload.

Usage (GPU): python tools/sweep_concurrency.py [--dtype fp32] [--batches 60] [--configs 4x3,6x4,...]
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="fp32")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--batches", type=int, default=60)
    ap.add_argument("--configs", default="4x3,2x2,3x3,5x4,6x4,6x3,8x4")
    ap.add_argument("--inputs", default="jpeg", choices=["rgb", "jpeg"], help="see tools/engine_probe.py")
    a = ap.parse_args(argv)
    import torch

    from bench import engine_throughput
    from inference_arena_amd.data.curator import DatasetManifest, load_manifest_images
    from inference_arena_amd.engine.pipeline import GpuPipeline
    from inference_arena_amd.models.zoo import default_models

    sfx = "" if a.dtype == "fp32" else f"_{a.dtype}"
    man = DatasetManifest.load(ROOT / "data" / "synthetic_set" / f"manifest_w0_n100{sfx}.json")
    images = load_manifest_images(man)
    models = default_models(0)
    jset = None
    if a.inputs == "jpeg":
        from inference_arena_amd.data.synthetic import encode_jpeg
        from inference_arena_amd.ops import native

        jset = native().JpegSet([encode_jpeg(im, 90) for im in images], pinned=True)
    torch.cuda.set_device(0)
    out = []
    for cfg in a.configs.split(","):
        slots, conc = (int(v) for v in cfg.split("x"))
        os.environ["ARENA_SLOTS"], os.environ["ARENA_CONCURRENCY"] = str(slots), str(conc)
        pipe = GpuPipeline(*models, device=0, buckets=[a.batch], dtype=a.dtype)
        engine_throughput(pipe.ex, images, a.batch, 10, jset)
        r = [engine_throughput(pipe.ex, images, a.batch, a.batches, jset) for _ in range(2)]
        row = {"slots": pipe.ex.num_slots(), "streams": conc, "req_s": [round(v, 1) for v in r]}
        print(json.dumps(row), flush=True)
        out.append(row)
        del pipe
        gc.collect()
        torch.cuda.synchronize()
    return 0


if __name__ == "__main__":
    sys.exit(main())
