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
    ap.add_argument("--s3", action="store_true",
                    help="first fetch the repository from the MinIO/S3 bucket (experiment.yaml infrastructure.minio, "
                         "MINIO_* env overrides) into --repository, like the reference's init containers")
    ap.add_argument("--bucket", default=None)
    a = ap.parse_args(argv)
    if a.s3:
        import os

        from inference_arena_amd.config import get_minio_config
        from inference_arena_amd.repository.s3 import S3Client, download_repository

        client = S3Client.from_config()
        bucket = a.bucket or os.environ.get("MINIO_BUCKET") or get_minio_config().get("bucket", "models")
        client.wait_ready(bucket)
        got = download_repository(client, bucket, a.repository)
        print(f"fetched {len(got)} object(s) from s3://{bucket} -> {a.repository}")
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
