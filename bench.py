#!/usr/bin/env python3
"""Headline benchmark: whole-node req/s + P50/P99 latency of the
YOLOv5n -> MobileNetV2 pipeline on 1..8 MI355X (BASELINE.json metric).

One process per GPU (torchrun for N > 1; RANK/LOCAL_RANK/WORLD_SIZE from the
environment).  Each rank:
  * builds the random-init networks and plans the native program; rank 0's
    folded weight blob is broadcast to every replica with RCCL over xGMI;
  * loads the curated synthetic workload (3-5 detections per image, mean 4:
    the reference's thesis test-set protocol, curated with the GPU pipeline
    itself and cached in data/synthetic_set/);
  * runs ``--warmup`` untimed steps, then exactly ``--steps`` timed steps
    bracketed by barrier + device synchronisation.  A step is one dynamic
    batch of ``--batch`` requests through the full device pipeline (host
    staging copy of the decoded RGB images, H2D, letterbox, 75 detector convs,
    decode, NMS, crop gather, 52 classifier layers, top-5, D2H, per-request
    result split).  As in the model server's instance loop, up to one batch
    per executor staging slot is in flight; every slot runs its hipGraph on
    its own stream and activation arena, so consecutive batches overlap on
    the device (the small 20x20 / 7x7 layers of one batch leave CUs free for
    the other) while the next batch's H2D copy streams in.
Rank 0 prints one JSON line; ``value`` is total requests/s over all ranks
(time = max over ranks), latencies are per-batch completion latencies.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from collections import deque
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = "req/sec (whole node) + P50/P99 e2e latency, YOLOv5n→MobileNetV2 at 1/2/4/8 GPU"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def load_workload(pipe, info, n_images: int, seed: int):
    from inference_arena_amd.data.curator import CurationConfig, DatasetManifest, curate, load_manifest_images
    from inference_arena_amd.parallel.dist import broadcast_object

    path = ROOT / "data" / "synthetic_set" / f"manifest_w{seed}_n{n_images}.json"
    man = None
    if info.is_main:
        if path.exists():
            man = DatasetManifest.load(path)
        else:
            t = time.time()

            def counter(imgs):
                return [len(r) for r in pipe.infer(imgs)]

            _, man = curate(counter, CurationConfig(target_count=n_images), log=log)
            man.config["weight_seed"] = seed
            try:
                man.save(path)
            except OSError:
                pass
            log(f"curated {len(man.images)} images in {time.time() - t:.1f}s: {man.statistics}")
    man = broadcast_object(man.to_dict() if man is not None else None, info)
    man = DatasetManifest(**man)
    return load_manifest_images(man), man


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=32, help="requests per dynamic batch per GPU (max_bs 32)")
    ap.add_argument("--seed", type=int, default=0, help="weight seed")
    ap.add_argument("--images", type=int, default=100, help="curated workload size")
    ap.add_argument("--bs1-requests", type=int, default=100, help="sequential bs=1 requests for the latency probe")
    ap.add_argument("--crop-cap", type=int, default=None,
                    help="crops per image one classification pass holds (default: experiment.yaml gpu.crop_cap_per_image)")
    a = ap.parse_args(argv)

    import torch

    from inference_arena_amd.engine.pipeline import GpuPipeline
    from inference_arena_amd.models.zoo import default_models
    from inference_arena_amd.parallel import dist as D

    info = D.init_from_env()
    if info.world != a.gpus:
        log(f"warning: --gpus {a.gpus} but WORLD_SIZE={info.world}; reporting n_gpus={info.world}")
    torch.cuda.set_device(info.local_rank)
    torch.set_num_threads(4)

    t0 = time.time()
    yolo, mnet = default_models(a.seed)
    buckets = sorted({1, a.batch})
    pipe = GpuPipeline(yolo, mnet, device=info.local_rank, buckets=buckets, crop_cap_per_image=a.crop_cap)
    blob = D.broadcast_blob(pipe.program.weights if info.is_main else None, info)
    if info.world > 1:
        if not np.array_equal(blob, pipe.program.weights):
            log("rank", info.rank, "replacing local weights with rank 0's broadcast blob")
        pipe.ex.set_weights(blob)
    log(f"[rank {info.rank}] pipeline ready in {time.time() - t0:.1f}s; arena MB per bucket "
        f"{ {b: round(v / 2**20, 1) for b, v in pipe.arena_bytes.items()} }")

    images, man = load_workload(pipe, info, a.images, a.seed)
    n = len(images)
    B = a.batch
    off = (info.rank * 37) % n

    def batch_at(step):
        s = (off + step * B) % n
        return [images[(s + i) % n] for i in range(B)]

    depth = pipe.ex.num_slots()  # batches in flight, as the model server's instance loop keeps them

    def run(steps, lat, crops):
        q = deque()
        for st in range(steps):
            imgs = batch_at(st)
            q.append((pipe.submit(imgs), time.perf_counter()))
            if len(q) == depth:
                slot, ts = q.popleft()
                res = pipe.collect(slot, B)
                lat.append(time.perf_counter() - ts)
                crops.append(sum(len(r) for r in res))
        while q:
            slot, ts = q.popleft()
            res = pipe.collect(slot, B)
            lat.append(time.perf_counter() - ts)
            crops.append(sum(len(r) for r in res))

    run(a.warmup, [], [])
    torch.cuda.synchronize()
    D.barrier(info)
    torch.cuda.synchronize()
    lat, crops = [], []
    t_start = time.perf_counter()
    run(a.steps, lat, crops)
    torch.cuda.synchronize()
    t_local = time.perf_counter() - t_start
    D.barrier(info)
    t_max = D.allreduce_max(t_local, info)

    # bs=1 latency probe (monolithic single-request path), rank 0 only
    bs1 = []
    if info.is_main and a.bs1_requests > 0:
        for i in range(5):
            pipe.infer([images[i % n]])
        for i in range(a.bs1_requests):
            ts = time.perf_counter()
            pipe.infer([images[i % n]])
            bs1.append(time.perf_counter() - ts)

    all_lat = D.allgather_floats(lat, info)
    all_crops = D.allgather_floats([float(c) for c in crops], info)
    D.barrier(info)
    if info.is_main:
        flat = np.asarray([x for l in all_lat for x in l]) * 1e3
        total_req = a.steps * B * info.world
        value = total_req / t_max
        fan = float(np.sum([x for l in all_crops for x in l]) / total_req)
        out = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "req/s",
            "n_gpus": info.world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(t_max / a.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic COCO-shaped RGB images (curated to 3-5 detections, mean fan-out "
                    f"{fan:.2f}); random-init YOLOv5nu + MobileNetV2 weights; host JPEG decode excluded",
            "config": {
                "model": "YOLOv5nu(640)->MobileNetV2(224)",
                "global_batch": B * info.world,
                "seq_len": None,
                "parallelism": f"dp{info.world}",
                "per_gpu_batch": B,
                "image_size": 640,
                "crop_size": 224,
                "workload": {"images": n, "distribution": man.distribution, "mean_detections":
                             man.statistics.get("mean_detections")},
            },
            "p50_ms": round(float(np.percentile(flat, 50)), 3),
            "p99_ms": round(float(np.percentile(flat, 99)), 3),
            "mean_crops_per_request": round(fan, 3),
            "conv_kernel_choice": {f"impl{k}": v for k, v in sorted(__import__("collections").Counter(
                c for c in pipe.ex.conv_choices(B) if c).items())},
            "bs1_p50_ms": round(float(np.percentile(bs1, 50)) * 1e3, 3) if bs1 else None,
            "bs1_p99_ms": round(float(np.percentile(bs1, 99)) * 1e3, 3) if bs1 else None,
        }
        print(json.dumps(out), flush=True)
    D.shutdown(info)
    return 0


if __name__ == "__main__":
    sys.exit(main())
