#!/usr/bin/env python3
"""Refresh the Grafana dashboards and reload the monitoring stack (reference:
infrastructure/scripts/update-dashboards.sh, which seds the current container ids into each dashboard and
restarts Grafana).  The arena's dashboards select series by labels (architecture, gpu, compose service
name), so nothing container-specific is rewritten: this validates every dashboard, points them at the
provisioned Prometheus datasource uid, and asks Prometheus and Grafana to reload.

    python scripts/update_dashboards.py --datasource-uid prometheus --reload
"""
from __future__ import annotations

import argparse
import json
import sys
import urllib.request
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
DASH = ROOT / "monitoring" / "grafana" / "dashboards"


def retarget(d: dict, uid: str) -> int:
    n = 0
    for p in d.get("panels", []):
        ds = p.get("datasource")
        if isinstance(ds, dict) and ds.get("type") == "prometheus" and ds.get("uid") != uid:
            ds["uid"] = uid
            n += 1
        for t in p.get("targets", []):
            tds = t.get("datasource")
            if isinstance(tds, dict) and tds.get("type") == "prometheus" and tds.get("uid") != uid:
                tds["uid"] = uid
                n += 1
    return n


def check(d: dict, name: str) -> list[str]:
    errs = []
    if not d.get("uid", "").startswith("inference-arena-"):  # the reference's uids: inference-arena-{mono,micro,triton}
        errs.append(f"{name}: uid {d.get('uid')!r} is not inference-arena-*")
    for p in d.get("panels", []):
        for t in p.get("targets", []):
            e = t.get("expr", "")
            if not e:
                errs.append(f"{name}/{p.get('title')}: empty query")
            if 'container_id="' in e:
                errs.append(f"{name}/{p.get('title')}: hard-coded container id")
    return errs


def _post(url: str) -> str:
    try:
        req = urllib.request.Request(url, data=b"", method="POST")
        with urllib.request.urlopen(req, timeout=5) as r:
            return f"{url}: {r.status}"
    except OSError as e:
        return f"{url}: {e}"


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--datasource-uid", default=None)
    ap.add_argument("--reload", action="store_true")
    ap.add_argument("--prometheus", default="http://127.0.0.1:9090")
    ap.add_argument("--grafana", default="http://admin:admin@127.0.0.1:3000")
    a = ap.parse_args(argv)
    errs = []
    for f in sorted(DASH.glob("*.json")):
        d = json.loads(f.read_text())
        errs += check(d, f.name)
        if a.datasource_uid and retarget(d, a.datasource_uid):
            f.write_text(json.dumps(d, indent=2) + "\n")
            print(f"{f.name}: datasource -> {a.datasource_uid}")
    for e in errs:
        print("ERROR", e)
    if a.reload:
        print(_post(a.prometheus + "/-/reload"))
        print(_post(a.grafana + "/api/admin/provisioning/dashboards/reload"))
    return 1 if errs else 0


if __name__ == "__main__":
    sys.exit(main())
