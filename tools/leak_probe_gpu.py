#!/usr/bin/env python3
"""Host memory growth of the GPU engine per batch (companion of tools/leak_probe.py, which found the host-only
serving path flat at ~20 B/request): RSS after each round of

  replay   hipGraphLaunch of the captured bucket graph + a stream sync (Executor.replay / synchronize)
  submit   Executor.submit + collect of decoded RGB frames (host pack, H2D, graph, D2H, result unpack)
  jpeg     Executor.submit_jpeg_set of split-decoded JPEG coefficient sets (the HTTP path's inputs)
  batcher  the native DynamicBatcher over the executor, one request per image

A flat RSS after the first round is healthy; a steady slope is a leak of that many bytes per batch.

usage: python tools/leak_probe_gpu.py [--modes replay,submit,jpeg,batcher] [--rounds 5] [--batches 400]
"""
from __future__ import annotations

import argparse
import os
import sys
import threading
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def rss_mb() -> float:
    with open(f"/proc/{os.getpid()}/status") as f:
        for line in f:
            if line.startswith("VmRSS:"):
                return int(line.split()[1]) / 1024.0
    return 0.0


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--modes", default="batcher,jpeg,submit,replay")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--batches", type=int, default=400)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--trim", action="store_true", help="malloc_trim after each round (fragmentation vs leak)")
    a = ap.parse_args(argv)

    import numpy as np

    from inference_arena_amd.data.synthetic import encode_jpeg, synthetic_images
    from inference_arena_amd.engine.registry import build_session
    from inference_arena_amd.models.zoo import default_models
    from inference_arena_amd.ops import native

    C = native()
    yolo, mnet = default_models(0)
    pipe = build_session("pipeline", yolo, mnet, device=0, buckets=[1, a.batch])
    imgs = [np.ascontiguousarray(i) for i in synthetic_images(a.batch, 3)]
    jset = C.JpegSet([encode_jpeg(i) for i in imgs], pinned=True)
    ex = pipe.ex

    def run(mode: str, n: int) -> None:
        if mode == "replay":
            for _ in range(n // 20):
                ex.replay(a.batch, 0, 20)
                ex.synchronize()
        elif mode == "submit":
            for _ in range(n):
                ex.collect(ex.submit(imgs))
        elif mode == "jpeg":
            for _ in range(n):
                ex.collect(ex.submit_jpeg_set(jset, list(range(a.batch))))
        elif mode == "batcher":
            b = C.DynamicBatcher([ex], {"max_batch": a.batch, "max_queue_delay_us": 200})
            sem = threading.Semaphore(0)
            for _ in range(n):
                for im in imgs:
                    b.enqueue(im, lambda r: sem.release())
                for _ in imgs:
                    sem.acquire()
            b.shutdown()

    for mode in a.modes.split(","):
        try:
            run(mode, 20)  # warm-up: pools and caches reach their working size
        except Exception as e:  # noqa: BLE001 - report and go on with the next mode
            print(f"{mode}: failed: {e}", flush=True)
            continue
        base = rss_mb()
        for r in range(a.rounds):
            t0 = time.perf_counter()
            run(mode, a.batches)
            m = rss_mb()
            if a.trim:
                C.malloc_trim()
                print(f"{mode} round {r}: after malloc_trim rss {rss_mb():.1f} MB", flush=True)
            print(f"{mode} round {r}: {a.batches} batches in {time.perf_counter() - t0:.2f} s, rss {m:.1f} MB, "
                  f"{(m - base) * 1024 * 1024 / ((r + 1) * a.batches):.0f} B/batch since warm-up", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
