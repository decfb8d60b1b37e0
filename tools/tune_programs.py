#!/usr/bin/env python3
"""Regenerate the persisted conv tuning table (engine/tuning.py) for the arena's programs on a GPU:
every program kind x dtype x batch bucket is autotuned once and stored (``--base`` seeds the output
with an existing table, so a partial run keeps the other entries).  Copy the result into
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
    ap.add_argument("--dtypes", default="fp32,bf16")
    ap.add_argument("--base", default=None, help="table to start from (default: empty)")
    ap.add_argument("--kinds", default="pipeline,detector,classifier,yolo_raw,mobilenet_raw",
                    help="program kinds to retune (the others keep their --base entries)")
    a = ap.parse_args(argv)
    if a.base:
        Path(a.out).parent.mkdir(parents=True, exist_ok=True)
        Path(a.out).write_text(Path(a.base).read_text())
    os.environ["ARENA_TUNING"] = "retune"
    os.environ["ARENA_TUNING_FILE"] = str(Path(a.out).resolve())
    from inference_arena_amd.engine.pipeline import GpuClassifier, GpuDetector, GpuPipeline, GpuTensorModel
    from inference_arena_amd.models.zoo import default_models

    y, m = default_models(0)
    bk = [int(b) for b in a.buckets.split(",")]
    for dt in a.dtypes.split(","):
        for name, make in (
                ("pipeline", lambda: GpuPipeline(y, m, device=0, buckets=bk, dtype=dt)),
                ("detector", lambda: GpuDetector(y, device=0, buckets=bk, dtype=dt)),
                ("classifier", lambda: GpuClassifier(m, device=0, buckets=[b for b in bk if b >= 4] + [64], dtype=dt)),
                ("yolo_raw", lambda: GpuTensorModel.yolo(y, device=0, buckets=bk, dtype=dt)),
                ("mobilenet_raw", lambda: GpuTensorModel.mobilenet(m, device=0, buckets=bk, dtype=dt))):
            if name not in a.kinds.split(","):
                continue
            r = make()
            print(dt, name, {B: sum(1 for c in r.ex.conv_choices(B) if c) for B in r.buckets}, flush=True)
            del r
    print("wrote", a.out)
    return 0


if __name__ == "__main__":
    sys.exit(main())
