"""Evaluate the performance hypotheses H1a-H1d of experiment.yaml from sweep summaries.

Input: rows of ``runner.summarize`` (with ``architecture``), averaged over
runs per (architecture, users).  Architecture keys follow the spec:
monolithic, microservices, triton (the arena model server + gateway).
"""
from __future__ import annotations

from collections import defaultdict

import numpy as np


def aggregate(rows: list[dict]) -> dict[str, dict[int, dict]]:
    acc: dict = defaultdict(lambda: defaultdict(list))
    for r in rows:
        acc[r["architecture"]][int(r["users"])].append(r)
    out: dict = {}
    for arch, levels in acc.items():
        out[arch] = {}
        for u, rs in levels.items():
            out[arch][u] = {k: float(np.nanmean([x[k] for x in rs]))
                            for k in ("p50_latency_ms", "p99_latency_ms", "throughput_rps", "error_rate_percent")}
    return out


def evaluate(rows: list[dict], tolerance: float = 0.20, saturation_ms: float = 500.0) -> dict[str, dict]:
    a = aggregate(rows)
    res: dict[str, dict] = {}
    arches = set(a)

    def lv(arch, pred):
        return sorted(u for u in a.get(arch, {}) if pred(u))

    if {"monolithic", "microservices", "triton"} <= arches:
        low = [u for u in lv("monolithic", lambda u: u <= 10) if u in a["microservices"] and u in a["triton"]]
        res["H1a"] = {"levels": low, "supported": bool(low) and all(
            a["monolithic"][u]["p99_latency_ms"] < min(a["microservices"][u]["p99_latency_ms"],
                                                      a["triton"][u]["p99_latency_ms"]) for u in low)}
    if {"monolithic", "microservices"} <= arches:
        low = [u for u in lv("monolithic", lambda u: u <= 10) if u in a["microservices"]]
        ratios = {u: (a["microservices"][u]["p99_latency_ms"] - a["monolithic"][u]["p99_latency_ms"])
                  / a["monolithic"][u]["p99_latency_ms"] for u in low}
        res["H1b"] = {"overhead": ratios, "supported": bool(ratios) and all(v < tolerance for v in ratios.values())}
    if {"triton", "microservices"} <= arches:
        high = [u for u in lv("triton", lambda u: u >= 50) if u in a["microservices"]]
        gaps = {u: (a["triton"][u]["p99_latency_ms"] - a["triton"][u]["p50_latency_ms"],
                    a["microservices"][u]["p99_latency_ms"] - a["microservices"][u]["p50_latency_ms"]) for u in high}
        res["H1c"] = {"gaps": gaps, "supported": bool(gaps) and all(t < m for t, m in gaps.values())}
    sat = {}
    for arch in arches:
        over = [u for u in sorted(a[arch]) if a[arch][u]["p99_latency_ms"] > saturation_ms]
        sat[arch] = over[0] if over else None
    res["H1d"] = {"saturation_users": sat,
                  "supported": bool(sat) and all(v is not None and v < 100 for v in sat.values())}
    return res
