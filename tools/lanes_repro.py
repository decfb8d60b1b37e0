#!/usr/bin/env python3
"""Head-lanes stress outside pytest (a segfault here must not take the test runner down with it).

The arm-B detection service's shape (server/service_backends.py GpuDetectorBackend): the detector-only program
(engine/plans.py plan_detector) with the default bucket set behind the native DynamicBatcher, JPEG uploads
through the split decoder (run_jpeg) from concurrent requests, optionally exporting frames into a device ring.
Runs the same requests through a lanes-off and a lanes-on detector and compares the detections.  The native
crash tracer (csrc/runtime/crash_trace.cpp) prints the faulting thread's stack if it dies.

usage: python tools/lanes_repro.py [--program detector|pipeline] [--users 1,2,10] [--rounds 20] [--export]
"""
from __future__ import annotations

import argparse
import asyncio
import os
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def _runner(kind: str, models, lanes: bool, buckets):
    from inference_arena_amd.engine.registry import build_session

    os.environ["ARENA_HEAD_LANES"] = "1" if lanes else "0"
    yolo, mnet = models
    if kind == "detector":
        return build_session("detector", yolo, device=0, buckets=buckets)
    return build_session("pipeline", yolo, mnet, device=0, buckets=buckets)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--program", default="detector", choices=["detector", "pipeline"])
    ap.add_argument("--users", default="1,2,10")
    ap.add_argument("--rounds", type=int, default=20)
    ap.add_argument("--max-batch", type=int, default=32)
    ap.add_argument("--seed", type=int, default=0, help="weight seed (the services' ARENA_WEIGHT_SEED)")
    ap.add_argument("--export", action="store_true", help="export each frame into a device ring (device transport)")
    a = ap.parse_args(argv)

    from inference_arena_amd.data.synthetic import encode_jpeg, synthetic_images
    from inference_arena_amd.models.zoo import default_models
    from inference_arena_amd.ops import native
    from inference_arena_amd.processing.transforms import load_image_from_bytes
    from inference_arena_amd.server.batching import AsyncBatcher
    from inference_arena_amd.server.service_backends import _default_buckets

    print("crash trace installed:", native().crash_trace_installed(), flush=True)
    models = default_models(a.seed)
    buckets = _default_buckets(a.max_batch)
    imgs = synthetic_images(24, 7) + synthetic_images(8, 8, hw=(480, 640))
    uploads = [encode_jpeg(im) for im in imgs]
    ring = None
    if a.export:
        from inference_arena_amd.server.device_transport import DeviceImageRing

        ring = DeviceImageRing(64, 640 * 640 * 3, device=0)

    async def decode(data):
        return load_image_from_bytes(data)

    def drive(runner, tag):
        b = AsyncBatcher([runner], max_batch=a.max_batch, max_queue_delay_us=500)
        out = {}

        async def one(i):
            slot = ring.acquire() if ring is not None else None
            try:
                d = await b.run_jpeg(uploads[i], decode, export_to=ring.slot_ptr(slot) if ring is not None else 0)
            finally:
                if slot is not None:
                    ring.release(slot)
            return d

        async def go():
            for users in [int(u) for u in a.users.split(",")]:
                t0 = time.perf_counter()
                lat = []
                for r in range(a.rounds):
                    idx = [(r * users + k) % len(uploads) for k in range(users)]
                    t1 = time.perf_counter()
                    res = await asyncio.gather(*(one(i) for i in idx))
                    lat.append((time.perf_counter() - t1) * 1e3)
                    for i, d in zip(idx, res):
                        out.setdefault((users, i), d)
                lat.sort()
                print(f"[{tag}] users {users}: {a.rounds} rounds in {time.perf_counter() - t0:.2f} s "
                      f"(batches {b.stats().get('batches')}); round latency P50 {lat[len(lat) // 2]:.3f} ms "
                      f"P90 {lat[int(len(lat) * 0.9)]:.3f} ms", flush=True)

        try:
            asyncio.run(go())
        finally:
            b.close()
        return out

    ref = drive(_runner(a.program, models, False, buckets), "lanes off")
    got = drive(_runner(a.program, models, True, buckets), "lanes on")
    bad = 0
    for k, d in ref.items():
        e = got[k]
        if d["det_count"] != e["det_count"] or not np.array_equal(d["det"], e["det"]):
            bad += 1
        if a.program == "pipeline" and not np.array_equal(d["topk_idx"], e["topk_idx"]):
            bad += 1
    print(f"compared {len(ref)} answers, {bad} mismatches; detections per image "
          f"{np.mean([d['det_count'] for d in ref.values()]):.1f}", flush=True)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
