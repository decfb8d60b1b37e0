"""experiment.yaml loader and typed accessors.

API-compatible with the reference's ``shared.config`` (src/shared/config.py:
get_config :57-80, reload_config :83-92, get_controlled_variable :100-138,
get_controlled_variables :141-162, get_model_config :170-187,
get_model_names :190-201, get_hypothesis :209-230,
get_hypotheses_by_category :233-254, get_infrastructure_config :262-287,
get_minio_config :290-303, get_triton_config :311-323,
get_load_testing_config :331-342, get_concurrent_user_levels :345-357,
get_metadata :365-377, get_spec_version :380-390, validate_config
:398-475), plus accessors for the additive ``gpu:`` section.

The file is located through ``ARENA_EXPERIMENT_YAML`` if set, else the
repository root, else the current directory.  YAML is parsed with the safe
loader only.
"""
from __future__ import annotations

import os
import threading
from pathlib import Path
from typing import Any

import yaml

_REPO_ROOT = Path(__file__).resolve().parent.parent
_lock = threading.Lock()
_cache: dict[str, Any] | None = None


def config_path() -> Path:
    env = os.environ.get("ARENA_EXPERIMENT_YAML")
    if env:
        return Path(env)
    for cand in (_REPO_ROOT / "experiment.yaml", Path.cwd() / "experiment.yaml"):
        if cand.exists():
            return cand
    return _REPO_ROOT / "experiment.yaml"


def _load() -> dict[str, Any]:
    p = config_path()
    if not p.exists():
        raise FileNotFoundError(f"experiment.yaml not found at {p}")
    with open(p, encoding="utf-8") as f:
        data = yaml.safe_load(f)
    if not isinstance(data, dict):
        raise ValueError(f"{p} does not contain a mapping")
    return data


def get_config() -> dict[str, Any]:
    """The parsed experiment specification (cached after the first call)."""
    global _cache
    with _lock:
        if _cache is None:
            _cache = _load()
        return _cache


def reload_config() -> dict[str, Any]:
    """Drop the cache and re-read the file."""
    global _cache
    with _lock:
        _cache = None
    return get_config()


def _section(cfg: dict[str, Any], key: str, where: str) -> Any:
    if key not in cfg:
        raise KeyError(f"'{key}' not found in {where}")
    return cfg[key]


def get_controlled_variables(section: str) -> dict[str, Any]:
    cv = _section(get_config(), "controlled_variables", "experiment.yaml")
    return _section(cv, section, "controlled_variables")


def get_controlled_variable(section: str, key: str) -> Any:
    return _section(get_controlled_variables(section), key, f"controlled_variables.{section}")


def get_model_config(model_name: str) -> dict[str, Any]:
    return _section(get_controlled_variables("models"), model_name, "controlled_variables.models")


def get_model_names() -> list[str]:
    return list(get_controlled_variables("models").keys())


def get_hypothesis(hypothesis_id: str) -> dict[str, Any]:
    return _section(_section(get_config(), "hypotheses", "experiment.yaml"), hypothesis_id, "hypotheses")


def get_hypotheses_by_category(category: str) -> dict[str, dict[str, Any]]:
    hs = get_config().get("hypotheses", {})
    return {k: v for k, v in hs.items() if v.get("category") == category}


def get_infrastructure_config(service: str | None = None) -> dict[str, Any]:
    infra = _section(get_config(), "infrastructure", "experiment.yaml")
    if service is None:
        return infra
    return _section(infra, service, "infrastructure")


def get_minio_config() -> dict[str, Any]:
    return get_infrastructure_config("minio")


def get_triton_config() -> dict[str, Any]:
    return _section(get_config(), "triton", "experiment.yaml")


def get_load_testing_config() -> dict[str, Any]:
    return get_controlled_variables("load_testing")


def get_concurrent_user_levels() -> list[int]:
    iv = _section(get_config(), "independent_variables", "experiment.yaml")
    return list(iv["concurrent_users"]["levels"])


def get_metadata() -> dict[str, Any]:
    return _section(get_config(), "metadata", "experiment.yaml")


def get_spec_version() -> str:
    return str(get_metadata().get("spec_version", "unknown"))


def get_gpu_config() -> dict[str, Any]:
    """The additive MI355X section (defaults when absent)."""
    dflt = {
        "arch": "gfx950",
        "replicas": [1],
        "dtype": "fp32",
        "batch_buckets": [1, 2, 4, 8, 16, 32],
        "crop_cap_per_image": 6,
        "max_det": 300,
        "weight_seed": 0,
        "fanout_target_mean": 4.0,
        "host_threads": 8,
        "ports": {},
    }
    dflt.update(get_config().get("gpu", {}) or {})
    return dflt


def get_cost_config() -> dict:
    """RQ2 cost model prices (``cost`` section; defaults when absent)."""
    c = get_config().get("cost") or {}
    return {"gpu_hour_usd": float(c.get("gpu_hour_usd", 0.0)), "vcpu_hour_usd": float(c.get("vcpu_hour_usd", 0.0))}


def validate_config() -> list[str]:
    """Schema check; returns a list of human-readable problems (empty = valid)."""
    try:
        cfg = get_config()
    except Exception as e:  # noqa: BLE001 - report, don't raise
        return [f"Failed to load config: {e}"]
    errors: list[str] = []
    for sec in ("metadata", "research_questions", "hypotheses", "independent_variables",
                "controlled_variables", "infrastructure"):
        if sec not in cfg:
            errors.append(f"Missing required section: {sec}")
    cv = cfg.get("controlled_variables", {}) or {}
    for sec in ("models", "preprocessing", "resources", "onnx_runtime", "dataset", "load_testing"):
        if sec not in cv:
            errors.append(f"Missing controlled_variables section: {sec}")
    models = cv.get("models", {}) or {}
    for name in ("yolov5n", "mobilenetv2"):
        m = models.get(name)
        if m is None:
            errors.append(f"Missing model configuration: {name}")
            continue
        for field in ("opset_version", "input", "output"):
            if field not in m:
                errors.append(f"Model {name} missing field: {field}")
    ort = cv.get("onnx_runtime", {}) or {}
    for field in ("intra_op_num_threads", "inter_op_num_threads"):
        if field not in ort:
            errors.append(f"Missing onnx_runtime field: {field}")
    for hid, h in (cfg.get("hypotheses", {}) or {}).items():
        for field in ("category", "statement", "rationale"):
            if field not in h:
                errors.append(f"Hypothesis {hid} missing required field: {field}")
        if "testable_prediction" not in h and "prediction" not in h:
            errors.append(f"Hypothesis {hid} missing testable_prediction or prediction")
    cost = cfg.get("cost")
    if cost is not None:
        for k in ("gpu_hour_usd", "vcpu_hour_usd"):
            v = cost.get(k)
            if not isinstance(v, (int, float)) or v < 0:
                errors.append(f"cost.{k} must be a non-negative number")
    gpu = cfg.get("gpu")
    if gpu is not None:
        buckets = gpu.get("batch_buckets", [])
        if not buckets or sorted(buckets) != list(buckets) or any(b <= 0 for b in buckets):
            errors.append("gpu.batch_buckets must be a non-empty ascending list of positive ints")
    return errors
