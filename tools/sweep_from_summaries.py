#!/usr/bin/env python3
"""Rebuild an arm's sweep CSV from its per-level summary JSONs (loadgen/runner.py writes ``<arch>_sweep.csv`` per
serving_sweep call, so a protocol split over several gpurun calls keeps only the last call's levels in it; the
``<arch>_u<users>_r<run>_summary.json`` files of every call survive).

usage: python tools/sweep_from_summaries.py DIR [--out NAME]   (default NAME: <arch>_sweep_L<levels>.csv)
"""
from __future__ import annotations

import argparse
import csv
import json
import re
import sys
from pathlib import Path


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    d = Path(a.dir)
    rows = []
    for f in d.glob("*_u*_r*_summary.json"):
        m = re.match(r"(.+)_u(\d+)_r(\d+)_summary\.json$", f.name)
        if not m:
            continue
        s = json.loads(f.read_text())
        s.pop("env", None)
        rows.append((int(m.group(2)), int(m.group(3)), s))
    if not rows:
        print(f"no summaries in {d}", file=sys.stderr)
        return 1
    rows.sort(key=lambda t: (t[0], t[1]))
    arch = rows[0][2].get("architecture", d.name)
    levels = sorted({u for u, _, _ in rows})
    out = d / (a.out or f"{arch}_sweep_L{'_'.join(map(str, levels))}.csv")
    fields = list(rows[0][2])
    with open(out, "w", newline="") as fh:
        w = csv.DictWriter(fh, fieldnames=fields, extrasaction="ignore")
        w.writeheader()
        for _, _, s in rows:
            w.writerow(s)
    print(out)
    return 0


if __name__ == "__main__":
    sys.exit(main())
