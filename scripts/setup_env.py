#!/usr/bin/env python3
"""Write a .env for the arena from .env.example (reference: scripts/setup_env.py — dev / prod / custom).

  dev     the template as is (local processes, default credentials)
  prod    fresh random MinIO / Grafana secrets, WARNING logs, container limits sized to the host
  custom  prompt for every key (interactive), or apply --set KEY=VALUE overrides

    python scripts/setup_env.py --mode prod --gpus 8
    python scripts/setup_env.py --mode custom --set ARENA_DTYPE=bf16 --set ARENA_MAX_BATCH=16
"""
from __future__ import annotations

import argparse
import os
import re
import secrets
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
LINE = re.compile(r"^([A-Z][A-Z0-9_]*)=(.*?)(\s+#.*)?$")


def render(template: str, values: dict[str, str]) -> str:
    out = []
    for ln in template.splitlines():
        m = LINE.match(ln)
        if m and m.group(1) in values:
            comment = m.group(3) or ""
            ln = f"{m.group(1)}={values[m.group(1)]}" + (f"  {comment.strip()}" if comment else "")
        out.append(ln)
    return "\n".join(out) + "\n"


def template_values(template: str) -> dict[str, str]:
    vals = {}
    for ln in template.splitlines():
        m = LINE.match(ln)
        if m:
            vals[m.group(1)] = m.group(2).strip()
    return vals


def preset(mode: str, gpus: int, cpus: int, mem_mb: int) -> dict[str, str]:
    if mode == "dev":
        return {}
    if mode == "prod":
        per = max(2, cpus // max(1, gpus))
        return {"LOG_LEVEL": "WARNING", "MINIO_ACCESS_KEY": "arena-" + secrets.token_hex(4),
                "MINIO_SECRET_KEY": secrets.token_urlsafe(24), "GRAFANA_ADMIN_PASSWORD": secrets.token_urlsafe(16),
                "GPUS": str(gpus), "LAST_GPU": str(gpus - 1), "CONTAINER_VCPU": str(per * gpus),
                "CONTAINER_MEMORY": str(max(4096, mem_mb // 2)), "ARENA_DECODE_THREADS": str(min(16, per))}
    return {}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--mode", default="dev", choices=["dev", "prod", "custom"])
    ap.add_argument("--out", default=str(ROOT / ".env"))
    ap.add_argument("--template", default=str(ROOT / ".env.example"))
    ap.add_argument("--gpus", type=int, default=8)
    ap.add_argument("--set", action="append", default=[], metavar="KEY=VALUE")
    ap.add_argument("--force", action="store_true")
    a = ap.parse_args(argv)
    out = Path(a.out)
    if out.exists() and not a.force:
        print(f"{out} exists (use --force to overwrite)")
        return 1
    tpl = Path(a.template).read_text()
    vals = template_values(tpl)
    try:
        mem_mb = os.sysconf("SC_PAGE_SIZE") * os.sysconf("SC_PHYS_PAGES") // 2**20
    except (ValueError, OSError):
        mem_mb = 65536
    upd = preset(a.mode, a.gpus, os.cpu_count() or 8, mem_mb)
    if a.mode == "custom" and not a.set and sys.stdin.isatty():
        for k, v in vals.items():
            ans = input(f"{k} [{v}]: ").strip()
            if ans:
                upd[k] = ans
    for kv in a.set:
        k, _, v = kv.partition("=")
        if k not in vals:
            print(f"unknown key {k} (not in the template)")
            return 2
        upd[k] = v
    out.write_text(render(tpl, upd))
    os.chmod(out, 0o600)
    print(f"wrote {out} ({a.mode}; {len(upd)} value(s) changed)")
    return 0


if __name__ == "__main__":
    sys.exit(main())
