"""Data / env / dashboard CLIs (reference: scripts/setup_data.py, scripts/setup_env.py,
infrastructure/scripts/update-dashboards.sh).  CPU only."""
from __future__ import annotations

import subprocess
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]


def _run(*args):
    return subprocess.run([sys.executable, *map(str, args)], capture_output=True, text=True, cwd=ROOT, timeout=600)


def test_setup_env_modes(tmp_path):
    out = tmp_path / ".env"
    r = _run(ROOT / "scripts" / "setup_env.py", "--mode", "prod", "--gpus", "4", "--out", out)
    assert r.returncode == 0, r.stderr
    text = out.read_text()
    assert "GPUS=4" in text and "LAST_GPU=3" in text and "LOG_LEVEL=WARNING" in text
    assert "MINIO_SECRET_KEY=minioadmin" not in text
    r = _run(ROOT / "scripts" / "setup_env.py", "--mode", "custom", "--set", "ARENA_DTYPE=bf16", "--out", out, "--force")
    assert r.returncode == 0 and "ARENA_DTYPE=bf16" in out.read_text()
    assert _run(ROOT / "scripts" / "setup_env.py", "--set", "NOPE=1", "--mode", "custom", "--out", out,
                "--force").returncode == 2


def test_update_dashboards_checks_pass():
    r = _run(ROOT / "scripts" / "update_dashboards.py")
    assert r.returncode == 0, r.stdout


def test_curate_paths_on_a_local_collection(tmp_path):
    """COCO-style curation over local files with a fake counter: 3-5 detections kept, 25/50/25 sample."""
    from PIL import Image

    from inference_arena_amd.data.curator import CurationConfig, curate_paths

    paths = []
    for i in range(60):
        p = tmp_path / f"{i:012d}.jpg"
        Image.fromarray(np.full((8, 8, 3), i, np.uint8)).save(p)
        paths.append(p)
    count = lambda imgs: [int(im[0, 0, 0]) % 7 for im in imgs]  # noqa: E731
    res, man = curate_paths(count, paths, CurationConfig(target_count=8), batch=16)
    assert man.statistics["total_images"] == 8
    assert all(3 <= r["detections"] <= 5 for r in man.images)
    assert res.total_scanned == 60 and res.skipped_low + res.skipped_high > 0
