"""scripts/validate_experiment.py — the deep experiment.yaml checks the validate-experiment-config workflow runs
(reference: .github/workflows/validate-experiment-config.yml)."""
from __future__ import annotations

import copy
import sys
from pathlib import Path

import yaml

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "scripts"))

import validate_experiment as V  # noqa: E402


def _cfg():
    return yaml.safe_load((ROOT / "experiment.yaml").read_text())


def test_repository_config_passes_every_check(tmp_path):
    rep = V.run(ROOT / "experiment.yaml")
    assert all(not v for k, v in rep.items() if not k.startswith("_")), rep
    md = V.markdown(rep)
    assert "validated" in md and "| programs | ok |" in md and "H1a" in md


def test_broken_configs_are_reported():
    c = _cfg()
    bad = copy.deepcopy(c)
    bad["controlled_variables"]["models"]["yolov5n"]["input"]["shape"] = [1, 3, 512, 512]
    assert V.check_models(bad) and V.check_preprocessing(bad)
    bad = copy.deepcopy(c)
    bad["controlled_variables"]["models"]["yolov5n"]["confidence_threshold"] = 1.5
    assert any("confidence_threshold" in e for e in V.check_models(bad))
    bad = copy.deepcopy(c)
    del bad["hypotheses"][next(iter(bad["hypotheses"]))]["statement"]
    assert V.check_hypotheses(bad)
    bad = copy.deepcopy(c)
    bad["gpu"]["batch_buckets"] = [32, 1]
    assert V.check_gpu(bad)
    bad = copy.deepcopy(c)
    bad["controlled_variables"]["onnx_runtime"]["intra_op_num_threads"] = 64
    assert V.check_threading(bad)
    bad = copy.deepcopy(c)
    bad["changelog"] = []
    assert V.check_changelog(bad, None)


def test_change_without_version_bump_is_flagged(tmp_path):
    c = _cfg()
    new = copy.deepcopy(c)
    new["controlled_variables"]["models"]["yolov5n"]["iou_threshold"] = 0.5
    assert any("spec_version" in e for e in V.check_changelog(new, c))
    keys = V.changed_keys(c, new)
    assert keys == ["controlled_variables.models.yolov5n.iou_threshold"]
    (tmp_path / "new.yaml").write_text(yaml.safe_dump(new))
    (tmp_path / "old.yaml").write_text(yaml.safe_dump(c))
    rep = V.run(tmp_path / "new.yaml", tmp_path / "old.yaml")
    assert rep["_changed"] == keys and rep["changelog"]
    assert "Changed keys" in V.markdown(rep)
