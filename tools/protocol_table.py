#!/usr/bin/env python3
"""Markdown table (mean ± sd over runs) of protocol summaries written by loadgen/runner.py.

usage: tools/protocol_table.py DIR[:LABEL] ...   (DIR holds <arch>_u<users>_r<run>_summary.json files)
Columns: arm, users, req/s, P50 ms, P99 ms, CPU % (all arm processes), runs, measurement seconds.  The
hypothesis checks (H1a-H1d) stay in scripts/analyze_results.py; this only renders the rows.
"""
from __future__ import annotations

import glob
import json
import statistics as st
import sys
from pathlib import Path


def rows(d: str, label: str | None = None) -> list[str]:
    by: dict[tuple[str, int], list[dict]] = {}
    for f in sorted(glob.glob(str(Path(d) / "*_u*_r*_summary.json"))):
        j = json.loads(Path(f).read_text())
        by.setdefault((j.get("architecture", "?"), int(j["users"])), []).append(j)
    out = []
    for (arch, users), runs in sorted(by.items()):
        def ms(k):
            v = [float(x[k]) for x in runs]
            return st.mean(v), (st.pstdev(v) if len(v) > 1 else 0.0)

        r, p50, p99 = ms("throughput_rps"), ms("p50_latency_ms"), ms("p99_latency_ms")
        cpu = st.mean(float(x.get("cpu_utilization_percent", 0.0)) for x in runs)
        secs = runs[0].get("measure_s", "")
        n = lambda v: f"{v:,.0f}".replace(",", " ")  # noqa: E731
        out.append(f"| {label or arch} | {users} | {n(r[0])} ± {n(r[1])} | {p50[0]:.1f} ± {p50[1]:.1f} | "
                   f"{p99[0]:.1f} ± {p99[1]:.1f} | {cpu:.0f} | {len(runs)} x {secs:g} s |")
    return out


def main(argv=None) -> int:
    args = sys.argv[1:] if argv is None else argv
    print("| arm | users | req/s | P50 ms | P99 ms | CPU % | runs |")
    print("|---|---|---|---|---|---|---|")
    for a in args:
        d, _, label = a.partition(":")
        for line in rows(d, label or None):
            print(line)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
