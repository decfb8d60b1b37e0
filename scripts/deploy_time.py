#!/usr/bin/env python3
"""RQ3 ``deployment_time_seconds`` (reference: /root/reference/experiment.yaml:55-61, H3c :160-164): launcher start
-> every service of the arm answering its health check, measured ``--runs`` times per arm with the arena's launcher
(scripts/start_arena.py, the counterpart of the reference's ``docker compose up`` + health checks).  Each run also
records the arm's idle resident memory right after it turned ready (H2c's ``baseline_memory_mb``: RSS of the
service processes and their children, in MiB).

    python scripts/deploy_time.py --arch monolithic microservices triton --runs 3 --out results/deploy_time.json
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "scripts"))


def tree_rss_mb(procs) -> float:
    import psutil

    total = 0
    seen = set()
    for p in procs:
        try:
            root = psutil.Process(p.pid)
            for q in [root] + root.children(recursive=True):
                if q.pid not in seen:
                    seen.add(q.pid)
                    total += q.memory_info().rss
        except psutil.Error:
            continue
    return total / 2**20


def measure(arch: str, runs: int, gpus: int, log_dir: Path, start=None, stop=None, settle_s: float = 2.0) -> dict:
    if start is None or stop is None:
        import start_arena

        start = start or start_arena.start
        stop = stop or start_arena.stop
    times, mems = [], []
    for r in range(runs):
        t0 = time.perf_counter()
        procs, ok = start(arch, gpus, log_dir / f"{arch}_run{r + 1}")
        dt = time.perf_counter() - t0
        try:
            if not ok:
                raise RuntimeError(f"{arch}: not ready (run {r + 1}); see {log_dir}")
            time.sleep(settle_s)
            mems.append(tree_rss_mb(procs))
        finally:
            stop(procs)
        times.append(dt)
        print(f"[deploy_time] {arch} run {r + 1}: ready in {dt:.2f} s, idle RSS {mems[-1]:.0f} MiB", flush=True)
        time.sleep(1.0)
    return {"deployment_time_seconds": statistics.mean(times), "runs": [round(t, 3) for t in times],
            "stdev_s": statistics.pstdev(times), "baseline_memory_mb": statistics.mean(mems),
            "baseline_memory_runs": [round(m, 1) for m in mems], "gpus": gpus}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--arch", nargs="+", default=["monolithic", "microservices", "triton"])
    ap.add_argument("--runs", type=int, default=3)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--logs", default="logs/deploy_time")
    ap.add_argument("--out", default="results/deploy_time.json")
    a = ap.parse_args(argv)
    out = {}
    for arch in a.arch:
        out[arch] = measure(arch, a.runs, a.gpus, Path(a.logs))
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    Path(a.out).write_text(json.dumps(out, indent=2) + "\n")
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main())
