#!/usr/bin/env python3
"""Init step of each topology (reference: architectures/*/init_*_models.py): copy models from the
repository into a service's model directory before it starts.

  --arch monolithic|microservices  flat <dst>/yolov5n.safetensors, <dst>/mobilenetv2.safetensors
  --arch triton                    full repository layout (versions, config.pbtxt, ensemble)
"""
from __future__ import annotations

import argparse
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main(argv=None) -> int:
    from inference_arena_amd.repository import init_flat, sync_repository, verify_repository

    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--arch", required=True, choices=["monolithic", "microservices", "triton"])
    ap.add_argument("--repository", default="model_repository")
    ap.add_argument("--dst", required=True)
    a = ap.parse_args(argv)
    bad = {k: v for k, v in verify_repository(a.repository).items() if v}
    if bad:
        print(f"repository problems: {bad}", file=sys.stderr)
        return 1
    if a.arch == "triton":
        n = len(sync_repository(a.repository, a.dst))
        print(f"copied {n} file(s) -> {a.dst}")
    else:
        for f in init_flat(a.repository, a.dst):
            print(f"-> {f}")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
