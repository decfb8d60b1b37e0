#!/usr/bin/env python3
"""Single-user latency breakdown: client-observed vs server-reported timing, per front-end path."""
from __future__ import annotations

import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "scripts"))


def probe(url: str, body: bytes, ctype: str, n: int = 20):
    import urllib.request

    import aiohttp
    import asyncio

    out = []
    for _ in range(n):
        t = time.perf_counter()
        req = urllib.request.Request(url, data=body, headers={"content-type": ctype})
        with urllib.request.urlopen(req, timeout=30) as r:
            js = json.loads(r.read())
        out.append(((time.perf_counter() - t) * 1e3, js["timing"]))

    async def aio():
        res = []
        async with aiohttp.ClientSession() as s:
            for _ in range(n):
                fd = aiohttp.FormData()
                fd.add_field("file", body_raw, filename="a.jpg", content_type="image/jpeg")
                t = time.perf_counter()
                async with s.post(url, data=fd) as r:
                    js = json.loads(await r.read())
                res.append(((time.perf_counter() - t) * 1e3, js["timing"]))
        return res

    body_raw = BODY_RAW
    a = asyncio.run(aio())
    return out, a


def main() -> int:
    from start_arena import start, stop

    from inference_arena_amd.data.curator import workload_images
    from inference_arena_amd.data.synthetic import encode_jpeg
    from inference_arena_amd.server.multipart import encode_multipart

    global BODY_RAW
    BODY_RAW = encode_jpeg(workload_images(1)[0], quality=95)
    body, ctype = encode_multipart("file", BODY_RAW)
    for arch, port in (("monolithic", 8100),):
        procs, ok = start(arch, 1, ROOT / "gpurun_out" / f"diag_{arch}")
        try:
            urllib_res, aio_res = probe(f"http://127.0.0.1:{port}/predict", body, ctype)
            for name, res in (("urllib", urllib_res), ("aiohttp", aio_res)):
                lat = sorted(r[0] for r in res)
                srv = sorted(r[1]["total_ms"] for r in res)
                print(f"{arch} {name}: client p50 {lat[len(lat)//2]:.2f} ms, server total p50 {srv[len(srv)//2]:.2f} ms; "
                      f"example timing {json.dumps(res[-1][1])}", flush=True)
        finally:
            stop(procs)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
