#!/usr/bin/env python3
"""Static bounds check of every executor program the arena can build (CI job; no GPU).

Plans the fused pipeline, the microservices detector / classifier, the split-topology stages and the
reference tensor contracts, in both precisions, and replays each against the layouts of every batch
bucket (engine/validate.py): a planner bug surfaces here as an exception instead of a GPU fault.
"""
from __future__ import annotations

import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main() -> int:
    from inference_arena_amd.config import get_gpu_config
    from inference_arena_amd.engine import plans
    from inference_arena_amd.engine.planner import layout
    from inference_arena_amd.engine.validate import validate_program
    from inference_arena_amd.models.zoo import default_models

    y, m = default_models(0)
    g = get_gpu_config()
    cap = int(g["crop_cap_per_image"])
    n = 0
    for dtype in ("fp32", "bf16"):
        progs = {
            "pipeline": plans.plan_pipeline(y, m, conf_thr=0.5, iou_thr=0.45, dtype=dtype),
            "detector": plans.plan_detector(y, conf_thr=0.5, iou_thr=0.45, dtype=dtype),
            "classifier": plans.plan_classifier(m, dtype=dtype),
            "split_detector": plans.plan_split_detector(y, conf_thr=0.5, iou_thr=0.45, dtype=dtype),
            "split_classifier": plans.plan_split_classifier(m, dtype=dtype),
            "yolo_raw": plans.plan_yolo_raw(y, dtype=dtype),
            "mobilenet_raw": plans.plan_mobilenet_raw(m, dtype=dtype),
        }
        for name, p in progs.items():
            for B in g["batch_buckets"]:
                cc = max(16, B * cap)
                validate_program(p, B, cc, max_det=int(g["max_det"]), cand_cap=8400,
                                 raw_out_bytes=int(p.meta.get("raw_out_bytes", 0)))
                _, total = layout(p.buffers, B, cc)
                n += 1
            print(f"{dtype:5s} {name:17s} ops {len(p.ops):4d}  weights {p.weights.nbytes / 2**20:6.2f} MiB  "
                  f"arena@{B} {total / 2**20:8.1f} MiB")
    print(f"ok: {n} (program, bucket) layouts validated")
    return 0


if __name__ == "__main__":
    sys.exit(main())
