#!/usr/bin/env python3
"""Regenerate the persisted conv tuning table (engine/tuning.py) for the arena's bf16 programs on a GPU:
every program kind x every batch bucket is autotuned once and stored.  Copy the result into
data/tuning/conv_tuning.json (``--out``) and commit it so every box captures the same kernels."""
from __future__ import annotations

import argparse
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--buckets", default="1,2,4,8,16,32")
    a = ap.parse_args(argv)
    os.environ["ARENA_TUNING"] = "retune"
    os.environ["ARENA_TUNING_FILE"] = str(Path(a.out).resolve())
    from inference_arena_amd.engine.pipeline import GpuClassifier, GpuDetector, GpuPipeline, GpuTensorModel
    from inference_arena_amd.models.zoo import default_models

    y, m = default_models(0)
    bk = [int(b) for b in a.buckets.split(",")]
    for name, make in (("pipeline", lambda: GpuPipeline(y, m, device=0, buckets=bk, dtype="bf16")),
                       ("detector", lambda: GpuDetector(y, device=0, buckets=bk, dtype="bf16")),
                       ("classifier", lambda: GpuClassifier(m, device=0, buckets=[b for b in bk if b >= 4] + [64],
                                                            dtype="bf16")),
                       ("yolo_raw", lambda: GpuTensorModel.yolo(y, device=0, buckets=bk, dtype="bf16")),
                       ("mobilenet_raw", lambda: GpuTensorModel.mobilenet(m, device=0, buckets=bk, dtype="bf16"))):
        r = make()
        print(name, {B: sum(1 for c in r.ex.conv_choices(B) if c) for B in r.buckets}, flush=True)
        del r
    print("wrote", a.out)
    return 0


if __name__ == "__main__":
    sys.exit(main())
