#!/usr/bin/env python3
"""Deep checks of experiment.yaml, the single source of truth (reference:
.github/workflows/validate-experiment-config.yml: syntax, required sections, model configs, preprocessing,
hypotheses, infrastructure, threading, changelog, tests, downstream impact, PR summary comment).

Every check is a function returning a list of problems; ``--markdown`` writes the PR-comment summary (the
workflow posts it); ``--base FILE`` compares against the previous experiment.yaml (changed keys, version bump,
downstream modules that read them).  Runs on CPU in seconds, locally as in CI:

    python scripts/validate_experiment.py [--base old_experiment.yaml] [--markdown summary.md]

Beyond the reference's checks, the arena's own consumers are exercised: the fp32 and bf16 programs are planned
from the configured models / thresholds / sizes and statically validated (engine/validate.py), and the GPU block
is checked against the model server's dynamic batching.
"""
from __future__ import annotations

import argparse
import json
import re
import subprocess
import sys
from pathlib import Path

import yaml

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

REQUIRED = ["metadata", "research_questions", "hypotheses", "independent_variables", "controlled_variables",
            "infrastructure", "triton", "gpu", "cost", "changelog"]
CONTROLLED = ["models", "preprocessing", "resources", "onnx_runtime", "dataset", "load_testing", "monitoring"]
SEMVER = re.compile(r"^\d+\.\d+\.\d+$")


def check_syntax(path: Path) -> tuple[dict, list[str]]:
    try:
        return yaml.safe_load(path.read_text()), []
    except yaml.YAMLError as e:
        return {}, [f"YAML syntax: {e}"]


def check_sections(c: dict) -> list[str]:
    errs = [f"missing top-level section '{k}'" for k in REQUIRED if k not in c]
    cv = c.get("controlled_variables", {})
    errs += [f"missing controlled_variables.{k}" for k in CONTROLLED if k not in cv]
    md = c.get("metadata", {})
    if not SEMVER.match(str(md.get("spec_version", ""))):
        errs.append(f"metadata.spec_version '{md.get('spec_version')}' is not semantic (X.Y.Z)")
    return errs


def check_models(c: dict) -> list[str]:
    errs = []
    models = c.get("controlled_variables", {}).get("models", {})
    want = {"yolov5n": ([1, 3, 640, 640], [1, 84, 8400]), "mobilenetv2": ([1, 3, 224, 224], [1, 1000])}
    for name, (ishape, oshape) in want.items():
        m = models.get(name)
        if m is None:
            errs.append(f"model '{name}' missing")
            continue
        if m.get("input", {}).get("shape") != ishape:
            errs.append(f"{name}: input shape {m.get('input', {}).get('shape')} != {ishape}")
        if m.get("output", {}).get("shape") != oshape:
            errs.append(f"{name}: output shape {m.get('output', {}).get('shape')} != {oshape}")
        for k in ("input", "output"):
            if m.get(k, {}).get("dtype") != "float32":
                errs.append(f"{name}: {k} dtype must stay float32 (the reference's ONNX graphs)")
    y = models.get("yolov5n", {})
    for k in ("confidence_threshold", "iou_threshold"):
        v = y.get(k)
        if not isinstance(v, (int, float)) or not 0.0 < float(v) < 1.0:
            errs.append(f"yolov5n.{k} = {v!r} must be in (0, 1)")
    return errs


def check_preprocessing(c: dict) -> list[str]:
    errs = []
    pp = c.get("controlled_variables", {}).get("preprocessing", {})
    models = c.get("controlled_variables", {}).get("models", {})
    yo, mb = pp.get("yolo", {}), pp.get("mobilenet", {})
    if yo.get("target_size") != models.get("yolov5n", {}).get("input", {}).get("shape", [0, 0, 0, 0])[-1]:
        errs.append("preprocessing.yolo.target_size must match the yolov5n input size")
    if mb.get("target_size") != models.get("mobilenetv2", {}).get("input", {}).get("shape", [0, 0, 0, 0])[-1]:
        errs.append("preprocessing.mobilenet.target_size must match the mobilenetv2 input size")
    if float(yo.get("normalization_scale", 0)) != 255.0:
        errs.append("preprocessing.yolo.normalization_scale must be 255")
    for k in ("mean", "std"):
        v = mb.get(k)
        if not (isinstance(v, list) and len(v) == 3 and all(0 < float(x) < 1 for x in v)):
            errs.append(f"preprocessing.mobilenet.{k} must be 3 values in (0, 1)")
    if (yo.get("target_size", 0) or 0) % 32:
        errs.append("preprocessing.yolo.target_size must be a multiple of 32 (stride-32 detector grid)")
    return errs


def check_hypotheses(c: dict) -> list[str]:
    errs = []
    hyp = c.get("hypotheses", {})
    if not hyp:
        return ["no hypotheses"]
    for hid, h in hyp.items():
        if not re.match(r"^H\d+[a-z]?$", hid):
            errs.append(f"hypothesis id '{hid}' is not H<n>[letter]")
        for k in ("category", "statement", "testable_prediction"):
            if not h.get(k):
                errs.append(f"{hid}: missing '{k}'")
        if h.get("category") not in ("performance", "scalability", "resource_efficiency", "operational_complexity",
                                     "cost"):
            errs.append(f"{hid}: unknown category {h.get('category')!r}")
    from inference_arena_amd.loadgen.hypotheses import evaluate  # every hypothesis must be evaluable
    try:
        evaluate([])
    except Exception as e:  # noqa: BLE001
        errs.append(f"hypothesis evaluator fails on an empty sweep: {e}")
    return errs


def check_infrastructure(c: dict) -> list[str]:
    errs = []
    res = c.get("controlled_variables", {}).get("resources", {})
    if int(res.get("vcpu_per_container", 0)) < 1:
        errs.append("resources.vcpu_per_container must be >= 1")
    if int(res.get("memory_mb_per_container", 0)) != int(res.get("memory_gb_per_container", 0)) * 1024:
        errs.append("resources.memory_mb_per_container must equal memory_gb_per_container * 1024")
    for arch in ("monolithic", "microservices", "triton"):
        a = res.get(arch, {})
        if a and a.get("total_vcpu") != a.get("containers", 0) * res.get("vcpu_per_container", 0):
            errs.append(f"resources.{arch}.total_vcpu != containers x vcpu_per_container")
    lt = c.get("controlled_variables", {}).get("load_testing", {})
    levels = lt.get("concurrent_users") or c.get("independent_variables", {}).get("concurrent_users", {}).get("levels")
    if levels is not None and (levels != sorted(levels) or levels[0] < 1):
        errs.append(f"user levels {levels} must be ascending and >= 1")
    return errs


def check_threading(c: dict) -> list[str]:
    errs = []
    ort = c.get("controlled_variables", {}).get("onnx_runtime", {})
    tr = c.get("triton", {}).get("parameters", {})
    if tr and str(tr.get("intra_op_thread_count")) != str(ort.get("intra_op_num_threads")):
        errs.append("triton.parameters.intra_op_thread_count must equal onnx_runtime.intra_op_num_threads")
    if int(ort.get("intra_op_num_threads", 0)) > int(c.get("controlled_variables", {}).get("resources", {})
                                                       .get("vcpu_per_container", 0)):
        errs.append("onnx_runtime.intra_op_num_threads exceeds the per-container vCPU budget")
    return errs


def check_gpu(c: dict) -> list[str]:
    errs = []
    g = c.get("gpu", {})
    if g.get("dtype") not in ("fp32", "bf16"):
        errs.append(f"gpu.dtype {g.get('dtype')!r} must be fp32 or bf16")
    b = g.get("batch_buckets", [])
    if not b or b != sorted(b):
        errs.append("gpu.batch_buckets must be ascending")
    mb = c.get("triton", {}).get("dynamic_batching", {}).get("max_batch_size")
    if b and mb is not None and b[-1] != mb:
        errs.append(f"gpu.batch_buckets[-1] {b[-1]} != triton.dynamic_batching.max_batch_size {mb}")
    return errs


def check_programs(c: dict) -> list[str]:
    """Plan the arena's programs from this configuration and validate them statically (no GPU)."""
    errs = []
    try:
        from inference_arena_amd.engine.plans import plan_pipeline
        from inference_arena_amd.engine.validate import validate_program
        from inference_arena_amd.models.zoo import default_models

        y = c["controlled_variables"]["models"]["yolov5n"]
        yolo, mnet = default_models(0)
        for dtype in ("fp32", "bf16"):
            prog = plan_pipeline(yolo, mnet, conf_thr=float(y["confidence_threshold"]),
                                 iou_thr=float(y["iou_threshold"]), dtype=dtype)
            for B in c.get("gpu", {}).get("batch_buckets", [1, 32]):
                validate_program(prog, B, 6 * B, max_det=300, cand_cap=8400)
    except Exception as e:  # noqa: BLE001
        errs.append(f"program planning / validation: {type(e).__name__}: {e}")
    return errs


def check_changelog(c: dict, base: dict | None) -> list[str]:
    errs = []
    log = c.get("changelog", [])
    if not isinstance(log, list) or not log:
        return ["changelog must be a non-empty list"]
    for i, e in enumerate(log):
        for k in ("date", "version", "change", "justification"):
            if not e.get(k):
                errs.append(f"changelog[{i}] missing '{k}'")
    ver = str(c.get("metadata", {}).get("spec_version"))
    if str(log[-1].get("version")) != ver and str(log[0].get("version")) != ver:
        errs.append(f"no changelog entry for spec_version {ver}")
    if base is not None and base != c:
        old = str(base.get("metadata", {}).get("spec_version"))
        if old == ver:
            errs.append(f"experiment.yaml changed but spec_version is still {ver} (bump it and add a changelog entry)")
    return errs


def changed_keys(old: dict, new: dict, prefix: str = "") -> list[str]:
    out = []
    for k in sorted(set(old) | set(new)):
        p = f"{prefix}.{k}" if prefix else str(k)
        a, b = old.get(k), new.get(k)
        if isinstance(a, dict) and isinstance(b, dict):
            out += changed_keys(a, b, p)
        elif a != b:
            out.append(p)
    return out


def downstream(keys: list[str]) -> dict[str, list[str]]:
    """Source files that read each changed top-level section (git grep of the section name)."""
    out = {}
    for sec in sorted({k.split(".")[0] for k in keys} | {".".join(k.split(".")[:2]) for k in keys}):
        name = sec.split(".")[-1]
        try:
            r = subprocess.run(["git", "grep", "-l", f"['\"]{name}['\"]", "--", "*.py"], cwd=ROOT,
                               capture_output=True, text=True, timeout=30)
            out[sec] = [f for f in r.stdout.split() if f][:12]
        except (OSError, subprocess.SubprocessError):
            out[sec] = []
    return out


def run(path: Path, base_path: Path | None = None) -> dict:
    c, errs = check_syntax(path)
    report = {"syntax": errs}
    base = None
    if base_path is not None and base_path.exists():
        base = yaml.safe_load(base_path.read_text())
    if c:
        report.update({
            "sections": check_sections(c), "models": check_models(c), "preprocessing": check_preprocessing(c),
            "hypotheses": check_hypotheses(c), "infrastructure": check_infrastructure(c),
            "threading": check_threading(c), "gpu": check_gpu(c), "programs": check_programs(c),
            "changelog": check_changelog(c, base),
        })
    keys = changed_keys(base, c) if base is not None and c else []
    report["_changed"] = keys
    report["_downstream"] = downstream(keys) if keys else {}
    report["_version"] = str(c.get("metadata", {}).get("spec_version")) if c else None
    report["_hypotheses"] = {k: v.get("statement", "") for k, v in c.get("hypotheses", {}).items()} if c else {}
    return report


def markdown(report: dict) -> str:
    ok = all(not v for k, v in report.items() if not k.startswith("_"))
    lines = [f"## Experiment configuration {'validated' if ok else 'has problems'} (spec {report['_version']})", "",
             "| check | result |", "|---|---|"]
    for k, v in report.items():
        if not k.startswith("_"):
            lines.append(f"| {k} | {'ok' if not v else '; '.join(v)} |")
    if report["_changed"]:
        lines += ["", "### Changed keys", ""] + [f"- `{k}`" for k in report["_changed"]]
        lines += ["", "### Downstream readers (review before merging)", ""]
        for sec, files in report["_downstream"].items():
            lines.append(f"- `{sec}`: " + (", ".join(f"`{f}`" for f in files) if files else "none found"))
    lines += ["", "### Hypotheses", ""] + [f"- **{k}**: {v}" for k, v in report["_hypotheses"].items()]
    return "\n".join(lines) + "\n"


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default=str(ROOT / "experiment.yaml"))
    ap.add_argument("--base", default=None, help="previous experiment.yaml (change detection, version bump)")
    ap.add_argument("--markdown", default=None, help="write the PR summary here")
    ap.add_argument("--json", default=None)
    a = ap.parse_args(argv)
    rep = run(Path(a.config), Path(a.base) if a.base else None)
    for k, v in rep.items():
        if not k.startswith("_"):
            print(f"[{'ok' if not v else 'FAIL'}] {k}" + ("" if not v else ": " + "; ".join(v)))
    if a.markdown:
        Path(a.markdown).write_text(markdown(rep))
    if a.json:
        Path(a.json).write_text(json.dumps(rep, indent=2) + "\n")
    return 0 if all(not v for k, v in rep.items() if not k.startswith("_")) else 1


if __name__ == "__main__":
    raise SystemExit(main())
