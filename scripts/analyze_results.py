#!/usr/bin/env python3
"""RQ1-RQ4 from loadgen sweep CSVs of one engine: hypothesis verdicts H1a-H1d (performance), H2a-H2d (resource
efficiency), H3a-H3c (operational complexity, with ``--deploy`` times from scripts/deploy_time.py), cost per 1000
requests per arm and level (experiment.yaml ``cost`` prices x GPUs + measured host CPU), the RQ3 LOC table and
the RQ4 crossover points and decision matrix (inference_arena_amd/analysis/decision.py).

    python scripts/analyze_results.py results/load/*_sweep.csv --deploy results/deploy_time.json --gpus 1 \
        --out results/analysis
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


def evaluate_h3_only(rq3, deploy):
    from inference_arena_amd.analysis.decision import evaluate_h3

    return evaluate_h3(rq3, deploy)


def main(argv=None) -> int:
    from inference_arena_amd.analysis import complexity_report, enrich_sweep_rows
    from inference_arena_amd.config import get_cost_config
    from inference_arena_amd.loadgen.hypotheses import evaluate

    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("sweeps", nargs="*")
    ap.add_argument("--gpus", type=int, default=1, help="GPUs the arms ran on (cost model)")
    ap.add_argument("--out", default="results/analysis")
    ap.add_argument("--deploy", default=None, help="scripts/deploy_time.py JSON (H3c, H2c idle memory)")
    a = ap.parse_args(argv)
    from inference_arena_amd.analysis.decision import analyze

    rows = [{k: _num(v) for k, v in r.items()} for f in a.sweeps for r in csv.DictReader(open(f))]
    rows = enrich_sweep_rows(rows, gpus=a.gpus, cost=get_cost_config())
    deploy = json.loads(Path(a.deploy).read_text()) if a.deploy else None
    rq3 = complexity_report()
    for arch, d in (deploy or {}).items():
        if arch in rq3:
            rq3[arch]["deployment_time_seconds"] = d.get("deployment_time_seconds")
    dec = analyze(rows, rq3, deploy) if rows else {"hypotheses": evaluate_h3_only(rq3, deploy), "rq4": {}}
    hyp = dict(evaluate(rows)) if rows else {}
    hyp.update(dec["hypotheses"])
    out = {"rq1_rq2_rows": rows, "hypotheses": hyp, "rq3": rq3, "rq4": dec.get("rq4", {})}
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
    if deploy:
        lines += ["", "| arch | deployment time s (mean of runs) | runs | idle RSS MiB |", "|---|---|---|---|"]
        for arm, dt in deploy.items():
            lines.append(f"| {arm} | {dt['deployment_time_seconds']:.2f} | {dt.get('runs')} | "
                         f"{dt.get('baseline_memory_mb', float('nan')):.0f} |")
    lines += ["", "| hypothesis | supported | evidence |", "|---|---|---|"]
    for h in sorted(hyp):
        ev = {k: v for k, v in hyp[h].items() if k != "supported"}
        lines.append(f"| {h} | {hyp[h].get('supported')} | {json.dumps(ev, default=str)[:300]} |")
    rq4 = out["rq4"]
    if rq4:
        lines += ["", "RQ4 crossover points:"]
        for c in rq4.get("crossover_points", []):
            lines.append(f"- {c['pair'][0]} vs {c['pair'][1]} on {c['metric']}: ~{c['users']} users "
                         f"({c['better_below']} better below, {c['better_above']} above)")
        if not rq4.get("crossover_points"):
            lines.append("- none: the arms keep their order over the measured levels")
        dm = rq4.get("decision_matrix", {})
        lines += ["", "| load regime | lowest P99 | highest req/s | lowest USD/1k | most req per CPU-s | lowest memory |",
                  "|---|---|---|---|---|---|"]
        for reg, row in dm.get("by_load_regime", {}).items():
            cell = lambda k: row.get(k, {}).get("best", "-")  # noqa: E731
            lines.append(f"| {reg} | {cell('lowest_p99_ms')} | {cell('highest_throughput_rps')} | "
                         f"{cell('lowest_cost_per_1000_usd')} | {cell('highest_requests_per_cpu_second')} | "
                         f"{cell('lowest_memory_mb')} |")
        lines += ["", "| P99 objective | best arm | max req/s per arm |", "|---|---|---|"]
        for slo, v in dm.get("by_p99_slo", {}).items():
            lines.append(f"| {slo} | {v['best']} | {v['max_throughput_rps']} |")
    (d / "summary.md").write_text("\n".join(lines) + "\n")
    print("\n".join(lines))
    return 0


if __name__ == "__main__":
    sys.exit(main())
