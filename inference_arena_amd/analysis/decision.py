"""RQ2-RQ4 hypothesis evaluation and the decision framework (reference: /root/reference/experiment.yaml:37-68,
116-164).  The reference pre-registers these hypotheses and metrics but ships no analysis code (its ``analysis/``
holds only ``.gitkeep``).  Inputs are the loadgen sweep rows (``runner.summarize``: throughput, P50/P99, CPU %
of the arm's process tree, RSS memory) averaged per (architecture, users), the RQ3 complexity report
(``rq.complexity_report``) and the measured deployment times (``scripts/deploy_time.py``).

Hypotheses (each returns the numbers it decided on and ``supported``):

* H2a  monolithic has the lowest resource consumption at all load levels.  Evaluated on the measured CPU use
       (``cpu_utilization_percent`` of each arm's processes) at every level all arms ran, and, as the reference
       states it, on the configured envelope (containers x vCPU from deploy/compose).
* H2b  microservices.requests_per_cpu_second < monolithic.requests_per_cpu_second (every common level);
       requests_per_cpu_second = throughput_rps / (cpu_utilization_percent / 100).
* H2c  triton.baseline_memory_mb > monolithic.baseline_memory_mb; baseline = idle RSS right after the arm turned
       ready (deploy_time records), else the memory at the lowest measured load level.
* H2d  the spread of efficiency across the arms shrinks as load grows (levels >= 50): the coefficient of variation
       of requests_per_cpu_second across arms is non-increasing from level to level.  (The variance of the raw
       values would mostly follow the mean throughput; the CV is the scale-free reading of "converges".)
* H3a  triton.application_code_loc < monolithic.application_code_loc
* H3b  microservices.total_config_loc > max(monolithic, triton)
* H3c  monolithic.deployment_time < min(microservices, triton)  (mean over runs of launcher start -> every
       service healthy)

RQ4:

* ``crossover_points``: for each pair of arms and each metric (throughput, P99), the user level where their
  order flips, linearly interpolated between the two measured levels that bracket the sign change;
* ``decision_matrix``: per load regime (low <= 10 users, mid 25-50, high >= 75) the best arm for lowest P99,
  highest throughput, lowest cost per 1000 requests, highest requests per CPU-second and lowest memory, and per
  P99 service-level objective the arm that sustains the most requests/s within it.
"""
from __future__ import annotations

import math
from collections import defaultdict
from statistics import mean, pstdev

ARCHES = ("monolithic", "microservices", "triton")
REGIMES = {"low (<= 10 users)": (0, 10), "mid (25-50 users)": (11, 50), "high (>= 75 users)": (51, 10 ** 9)}
SLOS_MS = (5.0, 10.0, 25.0, 50.0, 100.0, 500.0)
_KEYS = ("throughput_rps", "p50_latency_ms", "p99_latency_ms", "cpu_utilization_percent", "memory_usage_mb",
         "cost_per_1000_requests_usd", "error_rate_percent")


def _f(v) -> float:
    try:
        x = float(v)
    except (TypeError, ValueError):
        return math.nan
    return x


def levels(rows: list[dict]) -> dict[str, dict[int, dict]]:
    """{arch: {users: {metric: mean over runs}}} with requests_per_cpu_second derived."""
    acc: dict = defaultdict(lambda: defaultdict(list))
    for r in rows:
        acc[str(r["architecture"])][int(float(r["users"]))].append(r)
    out: dict = {}
    for arch, lv in acc.items():
        out[arch] = {}
        for u, rs in sorted(lv.items()):
            m = {}
            for k in _KEYS:
                vals = [_f(x.get(k)) for x in rs]
                vals = [v for v in vals if not math.isnan(v)]
                m[k] = mean(vals) if vals else math.nan
            cpu = m["cpu_utilization_percent"]
            m["requests_per_cpu_second"] = (m["throughput_rps"] / (cpu / 100.0)
                                            if cpu == cpu and cpu > 0 else math.nan)
            m["runs"] = len(rs)
            out[arch][u] = m
    return out


def _common(lv: dict, arches=ARCHES, pred=lambda u: True) -> list[int]:
    if not all(a in lv for a in arches):
        return []
    common = set.intersection(*(set(lv[a]) for a in arches))
    return sorted(u for u in common if pred(u))


def _configured_vcpus(root=None) -> dict[str, float]:
    """Containers x cpus limit per arm from deploy/compose (the reference's envelope, experiment.yaml:250-267)."""
    from pathlib import Path

    import yaml

    root = Path(root) if root else Path(__file__).resolve().parents[2]
    out = {}
    for arch in ARCHES:
        f = root / "deploy" / "compose" / f"{arch}.yml"
        if not f.exists():
            continue
        doc = yaml.safe_load(f.read_text()) or {}
        tot = 0.0
        for name, svc in (doc.get("services") or {}).items():
            lim = (((svc or {}).get("deploy") or {}).get("resources") or {}).get("limits") or {}
            cpus = lim.get("cpus")
            if cpus is None or "init" in str(name):
                continue
            s = str(cpus)
            if s.startswith("${") and ":-" in s:  # ${CONTAINER_VCPU:-2}
                s = s.split(":-", 1)[1].rstrip("}")
            try:
                tot += float(s)
            except ValueError:
                continue
        out[arch] = tot
    return out


def evaluate_h2(lv: dict, deploy: dict | None = None, root=None) -> dict:
    res: dict = {}
    common = _common(lv)
    if common:
        cpu = {u: {a: lv[a][u]["cpu_utilization_percent"] for a in ARCHES} for u in common}
        per_level = {u: bool(all(c[a] == c[a] for a in ARCHES) and c["monolithic"] <= min(c["microservices"],
                                                                                            c["triton"]))
                     for u, c in cpu.items()}
        conf = _configured_vcpus(root)
        res["H2a"] = {"measured_cpu_percent": cpu, "configured_vcpus": conf,
                      "supported_measured": all(per_level.values()),
                      "supported_configured": bool(conf) and conf.get("monolithic", math.inf) < min(
                          conf.get("microservices", 0), conf.get("triton", 0)),
                      "supported": all(per_level.values())}
    pair = _common(lv, ("monolithic", "microservices"))
    if pair:
        eff = {u: (lv["microservices"][u]["requests_per_cpu_second"], lv["monolithic"][u]["requests_per_cpu_second"])
               for u in pair}
        res["H2b"] = {"requests_per_cpu_second (micro, mono)": eff,
                      "supported": all(m < n for m, n in eff.values())}
    base = {}
    for a in ARCHES:
        d = (deploy or {}).get(a) or {}
        if d.get("baseline_memory_mb") is not None:
            base[a] = (float(d["baseline_memory_mb"]), "idle after ready")
        elif a in lv and lv[a]:
            u0 = min(lv[a])
            base[a] = (lv[a][u0]["memory_usage_mb"], f"{u0}-user level")
    if "triton" in base and "monolithic" in base:
        res["H2c"] = {"baseline_memory_mb": {a: round(v, 1) for a, (v, _) in base.items()},
                      "source": {a: s for a, (_, s) in base.items()},
                      "supported": base["triton"][0] > base["monolithic"][0]}
    high = _common(lv, pred=lambda u: u >= 50)
    if len(high) >= 2:
        cv = {}
        for u in high:
            e = [lv[a][u]["requests_per_cpu_second"] for a in ARCHES]
            e = [x for x in e if x == x]
            cv[u] = pstdev(e) / mean(e) if len(e) >= 2 and mean(e) > 0 else math.nan
        seq = [cv[u] for u in high]
        res["H2d"] = {"efficiency_cv_by_users": cv, "levels": high,
                      "supported": all(b <= a + 1e-12 for a, b in zip(seq, seq[1:]))}
    return res


def evaluate_h3(complexity: dict, deploy: dict | None = None) -> dict:
    res: dict = {}
    if all(a in complexity for a in ARCHES):
        app = {a: complexity[a]["application_code_loc"] for a in ARCHES}
        cfg = {a: complexity[a]["configuration_loc"] for a in ARCHES}
        res["H3a"] = {"application_code_loc": app, "supported": app["triton"] < app["monolithic"]}
        res["H3b"] = {"configuration_loc": cfg,
                      "supported": cfg["microservices"] > max(cfg["monolithic"], cfg["triton"])}
    if deploy and all(a in deploy and deploy[a].get("deployment_time_seconds") is not None for a in ARCHES):
        t = {a: float(deploy[a]["deployment_time_seconds"]) for a in ARCHES}
        res["H3c"] = {"deployment_time_seconds": t, "runs": {a: deploy[a].get("runs") for a in ARCHES},
                      "supported": t["monolithic"] < min(t["microservices"], t["triton"])}
    return res


def crossover_points(lv: dict, metrics=("throughput_rps", "p99_latency_ms")) -> list[dict]:
    """User levels where two arms swap order on a metric (linear interpolation inside the bracketing levels)."""
    out = []
    arches = [a for a in ARCHES if a in lv]
    for i, a in enumerate(arches):
        for b in arches[i + 1:]:
            us = _common(lv, (a, b))
            for m in metrics:
                d = [(u, lv[a][u][m] - lv[b][u][m]) for u in us if lv[a][u][m] == lv[a][u][m]
                     and lv[b][u][m] == lv[b][u][m]]
                for (u0, d0), (u1, d1) in zip(d, d[1:]):
                    if d0 == 0 or (d0 < 0) != (d1 < 0):
                        x = u0 if d0 == 0 else u0 + (u1 - u0) * (d0 / (d0 - d1))
                        better_hi = m == "throughput_rps"
                        lead_before = a if (d0 > 0) == better_hi else b
                        lead_after = b if lead_before == a else a
                        out.append({"pair": [a, b], "metric": m, "users": round(x, 1), "between": [u0, u1],
                                    "better_below": lead_before, "better_above": lead_after})
    return out


def decision_matrix(lv: dict) -> dict:
    arches = [a for a in ARCHES if a in lv]
    crit = {"lowest_p99_ms": ("p99_latency_ms", min), "highest_throughput_rps": ("throughput_rps", max),
            "lowest_cost_per_1000_usd": ("cost_per_1000_requests_usd", min),
            "highest_requests_per_cpu_second": ("requests_per_cpu_second", max),
            "lowest_memory_mb": ("memory_usage_mb", min)}
    regimes = {}
    for name, (lo, hi) in REGIMES.items():
        us = _common(lv, tuple(arches), lambda u: lo <= u <= hi)
        if not us:
            continue
        row = {"levels": us}
        for c, (m, pick) in crit.items():
            score = {a: mean([lv[a][u][m] for u in us]) for a in arches}
            score = {a: v for a, v in score.items() if v == v}
            if score:
                best = pick(score, key=score.get)
                row[c] = {"best": best, "values": {a: round(v, 6 if "cost" in c else 2) for a, v in score.items()}}
        regimes[name] = row
    slo = {}
    for s in SLOS_MS:
        cap = {}
        for a in arches:
            ok = [lv[a][u]["throughput_rps"] for u in lv[a] if lv[a][u]["p99_latency_ms"] <= s
                  and (lv[a][u]["error_rate_percent"] or 0) <= 1.0]
            cap[a] = max(ok) if ok else 0.0
        best = max(cap, key=cap.get) if any(cap.values()) else None
        slo[f"p99 <= {s:g} ms"] = {"max_throughput_rps": {a: round(v, 1) for a, v in cap.items()}, "best": best}
    return {"by_load_regime": regimes, "by_p99_slo": slo}


def analyze(rows: list[dict], complexity: dict | None = None, deploy: dict | None = None, root=None) -> dict:
    lv = levels(rows)
    out = {"levels": lv, "hypotheses": {}}
    out["hypotheses"].update(evaluate_h2(lv, deploy, root))
    if complexity is not None:
        out["hypotheses"].update(evaluate_h3(complexity, deploy))
    out["rq4"] = {"crossover_points": crossover_points(lv), "decision_matrix": decision_matrix(lv)}
    return out
