#!/usr/bin/env python3
"""Host memory growth of the native serving path per request, without a GPU.

The protocol summaries showed the arms' resident memory rising run after run (monolithic: ~1.3 KB per request over
a 60 s x 3 x 7-level sweep, profiles/protocol_r5/*_summary.json memory_usage_mb).  This drives the native HTTP front
end (split JPEG decoder threads, DynamicBatcher) over the host-only EchoInstance with the native closed-loop load
generator, in rounds, and prints the process's RSS after each round: a flat line after the first rounds (pools
and caches at their high-water mark) is healthy, a steady slope is a leak of that many bytes per request.

usage: python tools/leak_probe.py [--rounds 8] [--per-round 20000] [--users 32]
"""
from __future__ import annotations

import argparse
import io
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def rss_mb(pid: int | None = None) -> float:
    with open(f"/proc/{pid or os.getpid()}/status") as f:
        for line in f:
            if line.startswith("VmRSS:"):
                return int(line.split()[1]) / 1024.0
    return 0.0


def make_reqs(workload: bool = False) -> list[bytes]:
    """8 small multipart JPEG uploads (noise, 120-176 x 160, q90); ``workload``: the bench's 100 curated COCO-shaped
    frames as JPEG q90 (bench.py's uploads)"""
    import numpy as np
    from PIL import Image

    if workload:
        from inference_arena_amd.data.curator import DatasetManifest, load_manifest_images
        from inference_arena_amd.data.synthetic import encode_jpeg

        root = Path(__file__).resolve().parents[1]
        man = DatasetManifest.load(root / "data" / "synthetic_set" / "manifest_w0_n100.json")
        jpegs = [encode_jpeg(im, 90) for im in load_manifest_images(man)]
    else:
        rng = np.random.default_rng(0)
        jpegs = []
        for i in range(8):
            b = io.BytesIO()
            Image.fromarray((rng.random((120 + 8 * i, 160, 3)) * 255).astype(np.uint8)).save(b, "JPEG", quality=90)
            jpegs.append(b.getvalue())
    reqs = []
    for data in jpegs:
        bnd = "leakprobe"
        body = (f"--{bnd}\r\nContent-Disposition: form-data; name=\"file\"; filename=\"x.jpg\"\r\n"
                f"Content-Type: image/jpeg\r\n\r\n").encode() + data + f"\r\n--{bnd}--\r\n".encode()
        reqs.append((f"POST /predict HTTP/1.1\r\nHost: 127.0.0.1\r\nContent-Type: multipart/form-data; "
                     f"boundary={bnd}\r\nContent-Length: {len(body)}\r\n\r\n").encode() + body)
    return reqs


def load_only(port: int, n: int, users: int, workload: int = 0) -> int:
    """--load-only: the closed-loop load of one round from a process of its own (--external-load), so the probed
    process's RSS is the server's alone"""
    from inference_arena_amd.ops import native

    lg = native().HttpLoadGen({"host": "127.0.0.1", "port": port, "users": users, "threads": 2},
                              make_reqs(bool(workload)))
    lg.start()
    ok = lg.wait_completed(n, 600)
    lg.stop(30)
    print(lg.completed(), flush=True)
    return 0 if ok else 1


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--per-round", type=int, default=20000)
    ap.add_argument("--users", type=int, default=32)
    ap.add_argument("--decode-threads", type=int, default=4)
    ap.add_argument("--jpeg-host", action="store_true", help="with --gpu: reconstruct JPEGs on the host threads "
                    "(RGB inputs, no per-request coefficient DMA)")
    ap.add_argument("--jpeg-device", action="store_true", help="without --gpu: hand split-decoded coefficient sets to "
                    "the EchoInstance (the device-JPEG front-end branch, reconstructed on the host by the instance)")
    ap.add_argument("--gpu", action="store_true", help="the fused fp32 GPU pipeline instead of the host-only EchoInstance "
                    "(the monolithic server's exact path: split decoder, GPU reconstruction, executor)")
    ap.add_argument("--external-load", action="store_true", help="run each round's load generator in a child "
                    "process (the probed RSS is then the server's alone)")
    ap.add_argument("--workload", action="store_true", help="upload the bench's curated frames (JPEG q90, "
                    "COCO-shaped) instead of 8 small noise JPEGs")
    ap.add_argument("--load-only", nargs=4, type=int, metavar=("PORT", "N", "USERS", "WORKLOAD"), help=argparse.SUPPRESS)
    a = ap.parse_args(argv)
    if a.load_only:
        return load_only(*a.load_only)

    import numpy as np
    from PIL import Image

    from inference_arena_amd.ops import native
    from inference_arena_amd.server.native_front import NativeFrontEnd
    from inference_arena_amd.labels import load_labels

    C = native()
    if a.gpu:
        from inference_arena_amd.engine.registry import build_session
        from inference_arena_amd.models.zoo import default_models

        yolo, mnet = default_models(0)
        pipe = build_session("pipeline", yolo, mnet, device=0, buckets=[1, 2, 4, 8, 16, 32])
        inst = pipe.ex
    else:
        inst = C.EchoInstance(4, 32, 4, 500)
    batcher = C.DynamicBatcher([inst], {"max_batch": 32, "max_queue_delay_us": 300, "idle_queue_delay_us": 100})
    fe = NativeFrontEnd(batcher, load_labels(None), port=0, host="127.0.0.1", io_threads=2, decode_procs=1,
                        slots=64, decode_threads=a.decode_threads, jpeg_device=(a.gpu and not a.jpeg_host) or a.jpeg_device)
    reqs = make_reqs(a.workload)
    base = None
    done = 0
    try:
        for r in range(a.rounds):
            t0 = time.perf_counter()
            if a.external_load:
                import subprocess

                pr = subprocess.run([sys.executable, __file__, "--load-only", str(fe.port), str(a.per_round),
                                     str(a.users), str(int(a.workload))], capture_output=True, text=True, timeout=700)
                ok = pr.returncode == 0
                n = int(pr.stdout.split()[-1]) if pr.stdout.split() else 0
            else:
                lg = C.HttpLoadGen({"host": "127.0.0.1", "port": fe.port, "users": a.users, "threads": 2}, reqs)
                lg.start()
                ok = lg.wait_completed(a.per_round, 600)
                lg.stop(30)
                n = lg.completed()
                del lg  # its per-request records are freed with it
            done += n
            m = rss_mb()
            base = m if base is None else base
            mi = C.malloc_info()
            print(f"round {r}: {n} requests ({n / (time.perf_counter() - t0):.0f}/s), rss {m:.1f} MB, "
                  f"growth since round 0 {(m - base) * 1024 * 1024 / max(1, done - a.per_round):.0f} B/request; "
                  f"malloc: in use {mi['in_use'] / 2**20:.1f} MB, free {mi['free'] / 2**20:.1f} MB, "
                  f"chunk mmaps {mi['mmapped'] / 2**20:.1f} MB"
                  + ("" if ok else " (timeout)"), flush=True)
    finally:
        fe.close()
        batcher.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
