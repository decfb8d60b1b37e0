#!/usr/bin/env python3
"""Per-stage latency from the Prometheus scrapes a protocol sweep saves after every level
(loadgen/runner.py ``run_sweep(scrape=...)``: ``<arch>_u<users>_r<run>_metrics<i>.txt``).

The servers' histograms are cumulative over the process lifetime, so one level's share is the difference of
two consecutive scrapes.  For every ``*_seconds`` histogram series (e.g. ``arena_request_latency_seconds`` by
``stage``; the model server's KServe ``nv_inference_*`` durations are counters in microseconds and are reported
as means) this prints the count, mean and the P50 / P99 interpolated inside the histogram buckets.

usage: tools/stage_metrics.py AFTER.txt [BEFORE.txt]
"""
from __future__ import annotations

import re
import sys
from collections import defaultdict
from pathlib import Path

_LINE = re.compile(r'^([a-zA-Z_:][a-zA-Z0-9_:]*)(\{([^}]*)\})?\s+([-+0-9.eEinfNa]+)$')


def parse(path: str | None) -> dict[tuple[str, tuple], float]:
    out: dict[tuple[str, tuple], float] = {}
    if not path:
        return out
    for line in Path(path).read_text().splitlines():
        if not line or line.startswith("#"):
            continue
        m = _LINE.match(line.strip())
        if not m:
            continue
        labels = tuple(sorted(re.findall(r'(\w+)="([^"]*)"', m.group(3) or "")))
        try:
            out[(m.group(1), labels)] = float(m.group(4))
        except ValueError:
            continue
    return out


def _quantile(buckets: list[tuple[float, float]], q: float) -> float:
    """buckets: sorted (upper bound, cumulative count); linear interpolation inside the bucket."""
    total = buckets[-1][1]
    if total <= 0:
        return float("nan")
    target, prev_le, prev_c = q * total, 0.0, 0.0
    for le, c in buckets:
        if c >= target:
            if le == float("inf"):
                return prev_le
            frac = (target - prev_c) / (c - prev_c) if c > prev_c else 1.0
            return prev_le + frac * (le - prev_le)
        prev_le, prev_c = le, c
    return prev_le


def stages(after: str, before: str | None = None) -> list[dict]:
    a, b = parse(after), parse(before)
    d = {k: v - b.get(k, 0.0) for k, v in a.items()}
    hists: dict[tuple[str, tuple], list[tuple[float, float]]] = defaultdict(list)
    sums: dict[tuple[str, tuple], float] = {}
    counts: dict[tuple[str, tuple], float] = {}
    for (name, labels), v in d.items():
        if name.endswith("_seconds_bucket"):
            le = dict(labels).get("le", "+Inf")
            rest = tuple(x for x in labels if x[0] != "le")
            hists[(name[:-7], rest)].append((float("inf") if le == "+Inf" else float(le), v))
        elif name.endswith("_seconds_sum"):
            sums[(name[:-4], labels)] = v
        elif name.endswith("_seconds_count"):
            counts[(name[:-6], labels)] = v
    rows = []
    for key, bk in sorted(hists.items()):
        bk.sort()
        n = counts.get(key, bk[-1][1])
        if n <= 0:
            continue
        rows.append({"series": key[0], "labels": dict(key[1]), "count": int(n),
                     "mean_ms": 1e3 * sums.get(key, 0.0) / n, "p50_ms": 1e3 * _quantile(bk, 0.5),
                     "p99_ms": 1e3 * _quantile(bk, 0.99)})
    # KServe statistics counters (microseconds, cumulative): mean per request
    kv = defaultdict(dict)
    for (name, labels), v in d.items():
        base = name[:-6] if name.endswith("_total") else name  # prometheus_client names counters *_total
        if base.startswith("nv_inference_") and base.endswith("_duration_us"):
            kv[labels][base] = v
        elif base == "nv_inference_request_success":
            kv[labels]["n"] = v
    for labels, vals in kv.items():
        n = vals.get("n", 0.0)
        if n > 0:
            for name, v in sorted(vals.items()):
                if name != "n":
                    rows.append({"series": name, "labels": dict(labels), "count": int(n), "mean_ms": v / n / 1e3,
                                 "p50_ms": float("nan"), "p99_ms": float("nan")})
    return rows


def main(argv=None) -> int:
    args = sys.argv[1:] if argv is None else argv
    if not args:
        print(__doc__)
        return 2
    rows = stages(args[0], args[1] if len(args) > 1 else None)
    print("| series | labels | count | mean ms | P50 ms | P99 ms |")
    print("|---|---|---|---|---|---|")
    for r in rows:
        lab = ", ".join(f"{k}={v}" for k, v in r["labels"].items())
        print(f"| {r['series']} | {lab} | {r['count']} | {r['mean_ms']:.2f} | {r['p50_ms']:.2f} | {r['p99_ms']:.2f} |")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
