#!/usr/bin/env python3
"""RQ1-RQ3 summary from loadgen sweep CSVs: hypothesis verdicts (H1a-H1d), cost per 1000 requests per arm and
level (experiment.yaml ``cost`` prices x GPUs + measured host CPU), and the operational-complexity LOC table.

    python scripts/analyze_results.py results/load/*_sweep.csv --gpus 1 --out results/analysis
"""
from __future__ import annotations

import argparse
import csv
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def _num(v):
    try:
        return float(v)
    except (TypeError, ValueError):
        return v


def main(argv=None) -> int:
    from inference_arena_amd.analysis import complexity_report, enrich_sweep_rows
    from inference_arena_amd.config import get_cost_config
    from inference_arena_amd.loadgen.hypotheses import evaluate

    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("sweeps", nargs="*")
    ap.add_argument("--gpus", type=int, default=1, help="GPUs the arms ran on (cost model)")
    ap.add_argument("--out", default="results/analysis")
    a = ap.parse_args(argv)
    rows = [{k: _num(v) for k, v in r.items()} for f in a.sweeps for r in csv.DictReader(open(f))]
    rows = enrich_sweep_rows(rows, gpus=a.gpus, cost=get_cost_config())
    out = {"rq1_rq2_rows": rows, "hypotheses": evaluate(rows) if rows else {}, "rq3": complexity_report()}
    d = Path(a.out)
    d.mkdir(parents=True, exist_ok=True)
    (d / "summary.json").write_text(json.dumps(out, indent=2, default=str) + "\n")
    lines = ["| arch | users | req/s | P50 ms | P99 ms | CPU % | memory MB | USD / 1k req |", "|---|---|---|---|---|---|---|---|"]
    for r in rows:
        lines.append("| {} | {:.0f} | {:.1f} | {:.1f} | {:.1f} | {} | {} | {:.5f} |".format(
            r.get("architecture", "?"), r.get("users", 0), r.get("throughput_rps", 0.0), r.get("p50_latency_ms", 0.0),
            r.get("p99_latency_ms", 0.0), r.get("cpu_utilization_percent", "-"), r.get("memory_usage_mb", "-"),
            r["cost_per_1000_requests_usd"]))
    lines += ["", "| arch | application LOC | configuration LOC |", "|---|---|---|"]
    for arm in ("monolithic", "microservices", "triton"):
        c = out["rq3"][arm]
        lines.append(f"| {arm} | {c['application_code_loc']} | {c['configuration_loc']} |")
    lines.append(f"\nshared engine (kernels, runtime, planner): {out['rq3']['shared_engine_loc']} LOC")
    (d / "summary.md").write_text("\n".join(lines) + "\n")
    print("\n".join(lines))
    return 0


if __name__ == "__main__":
    sys.exit(main())
