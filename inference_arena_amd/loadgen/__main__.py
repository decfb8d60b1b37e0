"""CLI: ``python -m inference_arena_amd.loadgen --arch monolithic --url http://127.0.0.1:8100/predict``."""
from __future__ import annotations

import argparse
import json
from pathlib import Path


def main(argv=None) -> int:
    from ..config import get_concurrent_user_levels, get_load_testing_config
    from ..data.curator import workload_images
    from ..data.synthetic import encode_jpeg
    from .hypotheses import evaluate
    from .runner import LoadConfig, run_sweep

    lt = get_load_testing_config()
    ph = lt["phases"]
    ap = argparse.ArgumentParser(description="closed-loop load generator")
    ap.add_argument("--arch", default="monolithic", help="label: monolithic | microservices | triton")
    ap.add_argument("--url", default="http://127.0.0.1:8100/predict")
    ap.add_argument("--users", default=",".join(map(str, get_concurrent_user_levels())))
    ap.add_argument("--warmup", type=float, default=float(ph["warmup"]["duration_seconds"]))
    ap.add_argument("--measure", type=float, default=float(ph["measurement"]["duration_seconds"]))
    ap.add_argument("--cooldown", type=float, default=float(ph["cooldown"]["duration_seconds"]))
    ap.add_argument("--runs", type=int, default=int(lt["runs_per_configuration"]))
    ap.add_argument("--procs", type=int, default=1, help="client processes")
    ap.add_argument("--images", type=int, default=100, help="curated workload images to cycle through")
    ap.add_argument("--out", default="results/load")
    ap.add_argument("--evaluate", nargs="*", default=None, help="sweep CSVs to evaluate hypotheses over")
    ap.add_argument("--sample-ports", default="", help="comma list: sample CPU / memory of the processes "
                    "listening on these ports (and their children) during each level (RQ2)")
    ap.add_argument("--sample-pids", default="", help="comma list of server PIDs to sample (RQ2)")
    a = ap.parse_args(argv)
    if a.evaluate is not None:
        import csv

        rows = [dict(r) for f in a.evaluate for r in csv.DictReader(open(f))]
        for r in rows:
            for k in list(r):
                try:
                    r[k] = float(r[k])
                except ValueError:
                    pass
        print(json.dumps(evaluate(rows), indent=2, default=str))
        return 0
    images = [encode_jpeg(im, quality=95) for im in workload_images(a.images)]
    base = LoadConfig(url=a.url, warmup_s=a.warmup, measure_s=a.measure, cooldown_s=a.cooldown, procs=a.procs)
    users = [int(u) for u in a.users.split(",") if u]
    pids = [int(p) for p in a.sample_pids.split(",") if p]
    if a.sample_ports:
        from .resources import pids_listening_on

        pids += pids_listening_on([int(p) for p in a.sample_ports.split(",") if p])
    run_sweep(base, users, a.runs, images, Path(a.out), a.arch, sample_pids=sorted(set(pids)) or None)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
