#!/usr/bin/env python3
"""Populate (or verify) a model repository: <m>/1/model.safetensors, <m>/config.pbtxt,
<m>/metadata.json, the arena_pipeline ensemble and checksums.txt.

Reference: infrastructure/minio/init_models.py:446-542 (upload to MinIO with --force/--verify,
config.pbtxt from the generator, metadata.json with sha256).  The store here is a local or
shared filesystem path (``--repository``); ``--from`` syncs an existing repository instead of
exporting (the upload step of a two-host setup).
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main(argv=None) -> int:
    from inference_arena_amd.repository import build_repository, sync_repository, verify_repository

    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--repository", default="model_repository")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--verify", action="store_true", help="only verify the repository")
    ap.add_argument("--reference-compat", action="store_true",
                    help="configs exactly like the reference (max_batch_size 0, no dynamic batching)")
    ap.add_argument("--from", dest="src", default=None, help="copy this repository instead of exporting")
    ap.add_argument("--s3", action="store_true",
                    help="also upload the repository to the MinIO/S3 bucket of experiment.yaml infrastructure.minio "
                         "(MINIO_* env overrides; skip-if-present unless --force)")
    ap.add_argument("--bucket", default=None, help="bucket (default: infrastructure.minio.bucket / MINIO_BUCKET)")
    ap.add_argument("--endpoint", default=None, help="S3 endpoint host:port (default: MINIO_INTERNAL_ENDPOINT)")
    a = ap.parse_args(argv)
    if not a.verify:
        if a.src:
            copied = sync_repository(a.src, a.repository, force=a.force)
            print(f"synced {len(copied)} file(s) from {a.src}")
        else:
            rep = build_repository(a.repository, seed=a.seed, force=a.force, reference_compat=a.reference_compat)
            print(json.dumps(rep, indent=2))
    problems = verify_repository(a.repository)
    for name, p in problems.items():
        print(f"{name}: {'OK' if not p else '; '.join(p)}")
    if any(problems.values()):
        return 1
    if a.s3 and not a.verify:
        import os

        from inference_arena_amd.config import get_minio_config
        from inference_arena_amd.repository.s3 import S3Client, upload_repository

        client = S3Client.from_config(endpoint=a.endpoint)
        bucket = a.bucket or os.environ.get("MINIO_BUCKET") or get_minio_config().get("bucket", "models")
        client.wait_ready(bucket)
        done = upload_repository(a.repository, client, bucket, force=a.force)
        n_up = sum(1 for v in done.values() if v == "uploaded")
        print(f"s3://{bucket}: {n_up} uploaded, {len(done) - n_up} already present")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
