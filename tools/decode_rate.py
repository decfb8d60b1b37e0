#!/usr/bin/env python3
"""Host JPEG decode capacity of the multi-process decode pool (server/decode_pool.py) on this machine:
decodes/s for 1..N workers over the curated workload's JPEGs (no GPU)."""
from __future__ import annotations

import argparse
import sys
import threading
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--workers", default="1,4,8,15")
    ap.add_argument("--n", type=int, default=2000)
    ap.add_argument("--quality", type=int, default=90)
    a = ap.parse_args(argv)
    from inference_arena_amd.data.curator import workload_images
    from inference_arena_amd.data.synthetic import encode_jpeg
    from inference_arena_amd.server.decode_pool import ProcessDecodePool

    js = [encode_jpeg(im, a.quality) for im in workload_images(40, n_images=100)]
    for w in (int(x) for x in a.workers.split(",")):
        with ProcessDecodePool(workers=w, slots=256) as pool:
            sem = threading.Semaphore(0)
            cb = lambda tag, v, e: sem.release()  # noqa: E731
            for i in range(64):
                pool.submit(js[i % len(js)], i, cb)
            for _ in range(64):
                sem.acquire()
            t = time.perf_counter()
            inflight = 0
            for i in range(a.n):
                pool.submit(js[i % len(js)], i, cb)
                inflight += 1
                if inflight >= 200:
                    sem.acquire()
                    inflight -= 1
            for _ in range(inflight):
                sem.acquire()
            print(f"{w} workers: {a.n / (time.perf_counter() - t):.0f} decodes/s", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
