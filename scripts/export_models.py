#!/usr/bin/env python3
"""Export the arena's YOLOv5nu / MobileNetV2 weights (seeded random init, BN calibrated) as
safetensors with sha256 checksums.

Reference: scripts/export_models.py:106-207 (--force, --verify, --yolo-only, --mobilenet-only,
--output-dir; writes models/checksums.txt).  No pretrained downloads exist offline, so the
weights are the deterministic random-init networks of inference_arena_amd.models.zoo.
"""
from __future__ import annotations

import argparse
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main(argv=None) -> int:
    from inference_arena_amd.repository.store import export_model, load_module, sha256_file

    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--output-dir", default="models")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--verify", action="store_true", help="reload every exported file")
    g = ap.add_mutually_exclusive_group()
    g.add_argument("--yolo-only", action="store_true")
    g.add_argument("--mobilenet-only", action="store_true")
    a = ap.parse_args(argv)
    names = ["yolov5n"] if a.yolo_only else ["mobilenetv2"] if a.mobilenet_only else ["yolov5n", "mobilenetv2"]
    out = Path(a.output_dir)
    out.mkdir(parents=True, exist_ok=True)
    lines = []
    for n in names:
        f = out / f"{n}.safetensors"
        if f.exists() and not a.force:
            print(f"{n}: exists ({f}), use --force to overwrite")
        else:
            info = export_model(n, f, seed=a.seed)
            print(f"{n}: wrote {f} ({info['bytes'] / 2**20:.1f} MiB)")
        if a.verify:
            load_module(f, n)
            print(f"{n}: verified (loads into {n})")
        lines.append(f"{sha256_file(f)}  {f.name}")
    (out / "checksums.txt").write_text("\n".join(lines) + "\n")
    print(f"checksums -> {out / 'checksums.txt'}")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
