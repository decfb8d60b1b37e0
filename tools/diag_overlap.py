#!/usr/bin/env python3
"""Where does a bench step go?  Device-only graph replay (one slot vs both
slots on their own streams) against the host-side cost of ``submit`` (packing
32 decoded images into pinned staging + H2D enqueue) and ``collect``.

Usage (GPU): python tools/diag_overlap.py [--batch 32] [--iters 50]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args(argv)
    import numpy as np
    import torch

    from inference_arena_amd.data.curator import workload_images
    from inference_arena_amd.engine.pipeline import GpuPipeline
    from inference_arena_amd.models.zoo import default_models

    torch.cuda.set_device(0)
    yolo, mnet = default_models(0)
    B = a.batch
    pipe = GpuPipeline(yolo, mnet, device=0, buckets=[B])
    imgs = workload_images(B)
    out = {}
    # stage real inputs in both slots
    for _ in range(2):
        pipe.collect(pipe.submit(imgs), B)
        pipe.collect(pipe.submit(imgs), B)
    ex = pipe.ex

    def timed(fn, n):
        ex.synchronize()
        t = time.perf_counter()
        for _ in range(n):
            fn()
        ex.synchronize()
        return (time.perf_counter() - t) / n * 1e3

    out["replay_one_slot_ms"] = timed(lambda: ex.replay(B, 0, 1), a.iters)
    out["replay_two_slots_ms_per_graph"] = timed(lambda: (ex.replay(B, 0, 1), ex.replay(B, 1, 1)), a.iters) / 2
    ns = ex.num_slots()
    out["slots"] = ns
    out["replay_all_slots_ms_per_graph"] = timed(lambda: [ex.replay(B, s, 1) for s in range(ns)], a.iters) / ns
    # pipelined submit/collect with every slot in flight (what bench.py times)
    from collections import deque

    q = deque()
    ex.synchronize()
    t = time.perf_counter()
    for _ in range(a.iters):
        q.append(pipe.submit(imgs))
        if len(q) == ns:
            pipe.collect(q.popleft(), B)
    while q:
        pipe.collect(q.popleft(), B)
    out["pipelined_ms_per_batch"] = (time.perf_counter() - t) / a.iters * 1e3
    # host cost of submit (pack + enqueue) and collect (wait + unpack)
    sub, col = [], []
    for _ in range(a.iters):
        t0 = time.perf_counter()
        s = pipe.submit(imgs)
        t1 = time.perf_counter()
        pipe.collect(s, B)
        t2 = time.perf_counter()
        sub.append(t1 - t0)
        col.append(t2 - t1)
    out["submit_host_ms_p50"] = float(np.median(sub) * 1e3)
    out["collect_wait_ms_p50"] = float(np.median(col) * 1e3)
    out["image_bytes_per_batch_MB"] = sum(i.nbytes for i in imgs) / 2**20
    # raw H2D bandwidth from pinned memory (the executor's staging path), alone and under compute
    nb = sum(i.nbytes for i in imgs)
    src = torch.empty(nb, dtype=torch.uint8).pin_memory()
    dst = torch.empty(nb, dtype=torch.uint8, device="cuda")
    st = torch.cuda.Stream()
    for _ in range(3):
        with torch.cuda.stream(st):
            dst.copy_(src, non_blocking=True)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(st):
        e0.record(st)
        for _ in range(10):
            dst.copy_(src, non_blocking=True)
        e1.record(st)
    torch.cuda.synchronize()
    out["h2d_GBps_idle"] = nb * 10 / (e0.elapsed_time(e1) * 1e-3) / 1e9
    ex.replay(B, 1, 4)
    with torch.cuda.stream(st):
        e0.record(st)
        for _ in range(10):
            dst.copy_(src, non_blocking=True)
        e1.record(st)
    torch.cuda.synchronize()
    ex.synchronize()
    out["h2d_GBps_under_compute"] = nb * 10 / (e0.elapsed_time(e1) * 1e-3) / 1e9
    print(json.dumps({k: round(v, 3) for k, v in out.items()}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
