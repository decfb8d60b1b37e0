#!/usr/bin/env python3
"""Closed-loop HTTP load sweep over the three topologies on this node (fills BASELINE.md rows).

For each arch: start its services (scripts/start_arena.py), run the load generator at the given
user levels with short phases, stop the services.  Results (per-level CSV/JSON, sweep CSV,
hypothesis evaluation) go to --out.
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "scripts"))


def main(argv=None) -> int:
    from start_arena import start, stop

    from inference_arena_amd.data.curator import workload_images
    from inference_arena_amd.data.synthetic import encode_jpeg
    from inference_arena_amd.loadgen.hypotheses import evaluate
    from inference_arena_amd.loadgen.runner import LoadConfig, run_sweep

    ap = argparse.ArgumentParser()
    ap.add_argument("--archs", default="monolithic,microservices,triton")
    ap.add_argument("--users", default="1,10,50,100")
    ap.add_argument("--warmup", type=float, default=5)
    ap.add_argument("--measure", type=float, default=15)
    ap.add_argument("--cooldown", type=float, default=1)
    ap.add_argument("--runs", type=int, default=1)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--procs", type=int, default=4)
    ap.add_argument("--device", default="gpu")
    ap.add_argument("--out", default="gpurun_out/load")
    ap.add_argument("--procs-per-gpu", type=int, default=1)
    a = ap.parse_args(argv)
    out = Path(a.out)
    images = [encode_jpeg(im, quality=95) for im in workload_images(100)]
    ports = {"monolithic": 8100, "microservices": 8200, "triton": 8300}
    rows = []
    for arch in a.archs.split(","):
        procs, ok = start(arch, a.gpus, out / f"logs_{arch}", a.device, procs_per_gpu=a.procs_per_gpu)
        try:
            if not ok:
                print(f"{arch}: failed to start", flush=True)
                continue
            base = LoadConfig(url=f"http://127.0.0.1:{ports[arch]}/predict", warmup_s=a.warmup, measure_s=a.measure,
                              cooldown_s=a.cooldown, procs=a.procs)
            # RQ2: CPU % / memory of the arm's processes (and children: replicas, decode workers) per level
            pids = [p.pid for p in procs if getattr(p, "pid", None)]
            # the servers' own stage histograms (cumulative: diff consecutive levels); triton: the gateway and the
            # model server's KServe metrics port
            scrape = [f"http://127.0.0.1:{ports[arch]}/metrics"] + (["http://127.0.0.1:8002/metrics"]
                                                                    if arch == "triton" else [])
            rows += run_sweep(base, [int(u) for u in a.users.split(",")], a.runs, images, out, arch,
                              log=lambda *x: print(*x, flush=True), sample_pids=pids or None, scrape=scrape)
        finally:
            stop(procs)
    (out / "hypotheses.json").write_text(json.dumps(evaluate(rows), indent=2, default=str) + "\n")
    if rows:  # RQ2 cost per 1000 requests + RQ3 complexity (inference_arena_amd/analysis)
        from inference_arena_amd.analysis import complexity_report, enrich_sweep_rows
        from inference_arena_amd.config import get_cost_config

        rq = {"rows": enrich_sweep_rows(rows, gpus=a.gpus, cost=get_cost_config()), "rq3": complexity_report()}
        (out / "rq2_rq3.json").write_text(json.dumps(rq, indent=2, default=str) + "\n")
    print(json.dumps(evaluate(rows), default=str))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
