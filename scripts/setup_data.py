#!/usr/bin/env python3
"""Create the curated workload (reference: scripts/setup_data.py — download COCO val2017, curate
3-5-detection images at conf 0.5 / IoU 0.45, 25/50/25 balanced sample with seed 42, manifest.json).

Sources (no network here: COCO is read from a local directory or archive):
  synthetic  the arena's deterministic synthetic COCO-shaped stream (default; what bench.py uses)
  coco       a local val2017 tree (--coco-dir) or zip (--archive)
Counter devices: gpu (the device pipeline of --dtype) or cpu (the fp32 torch reference detector).

    python scripts/setup_data.py --out data/synthetic_set/manifest_w0_n100.json
    python scripts/setup_data.py --source coco --coco-dir data/coco --out data/thesis_test_set/manifest.json
"""
from __future__ import annotations

import argparse
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def make_counter(device: str, dtype: str, seed: int, jpeg_quality: int):
    from inference_arena_amd.config import get_model_config
    from inference_arena_amd.data.synthetic import encode_jpeg
    from inference_arena_amd.models.zoo import default_models
    from inference_arena_amd.processing.transforms import load_image_from_bytes

    y = get_model_config("yolov5n")
    yolo, mnet = default_models(seed)
    if device == "gpu":
        from inference_arena_amd.engine.pipeline import GpuDetector

        det = GpuDetector(yolo, device=0, buckets=[32], dtype=dtype)
        run = lambda imgs: [len(r) for r in det.infer(imgs)]  # noqa: E731
    else:
        from inference_arena_amd.engine.reference import ReferencePipeline

        ref = ReferencePipeline(yolo, mnet, conf_thr=float(y["confidence_threshold"]),
                                iou_thr=float(y["iou_threshold"]))
        run = lambda imgs: [len(ref.detect(im)) for im in imgs]  # noqa: E731

    def count(imgs):
        if jpeg_quality > 0:  # count on the uploads the load generator sends
            imgs = [load_image_from_bytes(encode_jpeg(im, jpeg_quality)) for im in imgs]
        return run(imgs)

    return count


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--source", default="synthetic", choices=["synthetic", "coco"])
    ap.add_argument("--coco-dir", default="data/coco")
    ap.add_argument("--archive", default=None, help="local val2017 zip to extract into --coco-dir")
    ap.add_argument("--out", required=True)
    ap.add_argument("--n", type=int, default=100)
    ap.add_argument("--device", default="gpu", choices=["gpu", "cpu"])
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--seed", type=int, default=0, help="weight seed")
    ap.add_argument("--jpeg-quality", type=int, default=90, help="synthetic: count on JPEG round trips (0: raw)")
    ap.add_argument("--limit", type=int, default=None, help="coco: scan at most this many files")
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--coco-url", default="http://images.cocodataset.org/zips/val2017.zip",
                    help="coco: where to fetch val2017.zip when no --archive exists ('' = never download)")
    a = ap.parse_args(argv)
    out = Path(a.out)
    if out.exists() and not a.force:
        print(f"{out} exists (use --force to re-curate)")
        return 0
    from inference_arena_amd.config import get_controlled_variables
    from inference_arena_amd.data.curator import CurationConfig, curate, curate_paths

    ds = get_controlled_variables("dataset")
    cfg = CurationConfig(target_count=a.n, min_detections=int(ds["detection_range"]["min"]),
                         max_detections=int(ds["detection_range"]["max"]), random_seed=int(ds["random_seed"]))
    log = lambda *x: print(*x, file=sys.stderr)  # noqa: E731
    t = time.time()
    if a.source == "synthetic":
        _, man = curate(make_counter(a.device, a.dtype, a.seed, a.jpeg_quality), cfg, log=log)
        man.config.update({"weight_seed": a.seed, "dtype": a.dtype, "jpeg_quality": a.jpeg_quality})
    else:
        from inference_arena_amd.data.coco import download_coco_val2017, get_coco_image_paths

        download_coco_val2017(a.coco_dir, archive=a.archive, url=a.coco_url or None)
        paths = get_coco_image_paths(a.coco_dir)[: a.limit]
        _, man = curate_paths(make_counter(a.device, a.dtype, a.seed, 0), paths, cfg, log=log)
        man.config.update({"weight_seed": a.seed, "dtype": a.dtype})
    man.save(out)
    print(f"curated {len(man.images)} images in {time.time() - t:.1f}s: {man.statistics} -> {out}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
