"""tools/sweep_from_summaries.py: a protocol split over several gpurun calls keeps only the last call's levels in
``<arch>_sweep.csv``; the per-level summaries of every call rebuild the whole sweep, ordered by users and run."""
from __future__ import annotations

import csv
import importlib.util
import json
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def test_rebuilds_every_level_in_order(tmp_path):
    spec = importlib.util.spec_from_file_location("sfs", ROOT / "tools" / "sweep_from_summaries.py")
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    for users in (50, 1, 10):
        for run in (2, 1):
            s = {"users": users, "requests": 100 * users + run, "throughput_rps": 1.5 * users,
                 "architecture": "monolithic", "run": run, "env": {"ARENA_X": "1"}}
            (tmp_path / f"monolithic_u{users}_r{run}_summary.json").write_text(json.dumps(s))
    assert m.main([str(tmp_path)]) == 0
    out = tmp_path / "monolithic_sweep_L1_10_50.csv"
    rows = list(csv.DictReader(open(out)))
    assert [(int(r["users"]), int(r["run"])) for r in rows] == [(1, 1), (1, 2), (10, 1), (10, 2), (50, 1), (50, 2)]
    assert "env" not in rows[0]
