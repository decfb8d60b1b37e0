"""Model repository: export, layout, checksums, verification, sync, init.

Reference equivalents
  * export with sha256 checksums ...... src/shared/model/exporter.py:72-92,
                                        scripts/export_models.py:106-207
  * repository upload (<m>/1/model.*, <m>/config.pbtxt, <m>/metadata.json;
    skip-if-present unless --force, --verify) .. infrastructure/minio/
                                        init_models.py:116-405
  * init containers (flat files for the custom services, full layout for
    the model server) ................... architectures/*/init_*_models.py

Layout (same as the reference's bucket / Triton repository)::

    <root>/<model>/config.pbtxt
    <root>/<model>/metadata.json        schema + sha256 + provenance
    <root>/<model>/<version>/model.safetensors
    <root>/arena_pipeline/config.pbtxt  ensemble (fused on the device)
    <root>/arena_pipeline/1/

Weights are safetensors (torch state_dict of the unfolded network, loaded
without executing anything from the file).  The repository lives on a local
or shared filesystem (``sync`` copies between two repositories) and can be
pushed to / pulled from a MinIO or S3 bucket with the same keys
(``repository/s3.py``: SigV4-signed REST, no SDK).
"""
from __future__ import annotations

import hashlib
import json
import shutil
import time
from dataclasses import dataclass
from pathlib import Path

from . import model_config as mc

MODEL_FILE = "model.safetensors"
ARCHS = {"yolov5n": "yolov5nu", "mobilenetv2": "mobilenetv2"}
PIPELINE = "arena_pipeline"


def sha256_file(path: Path, chunk: int = 1 << 20) -> str:
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for b in iter(lambda: f.read(chunk), b""):
            h.update(b)
    return h.hexdigest()


def _build_module(name: str, seed: int):
    from ..models.zoo import default_models

    yolo, mnet = default_models(seed)
    return yolo if ARCHS[name] == "yolov5nu" else mnet


def export_model(name: str, out_path: Path, *, seed: int = 0) -> dict:
    """Write ``name``'s weights (seeded random init, BN calibrated) as safetensors."""
    from safetensors.torch import save_file

    if name not in ARCHS:
        raise KeyError(f"unknown model '{name}' (known: {sorted(ARCHS)})")
    m = _build_module(name, seed)
    sd = {k: v.detach().contiguous().cpu() for k, v in m.state_dict().items()}
    out_path.parent.mkdir(parents=True, exist_ok=True)
    save_file(sd, str(out_path), metadata={"arch": ARCHS[name], "weight_seed": str(seed), "model": name})
    return {"path": str(out_path), "sha256": sha256_file(out_path), "bytes": out_path.stat().st_size}


def load_module(path: Path, name: str | None = None):
    """safetensors -> torch module of the recorded architecture (eval mode)."""
    from safetensors import safe_open
    from safetensors.torch import load_file

    from ..models.mobilenetv2 import MobileNetV2
    from ..models.yolov5nu import YOLOv5nu

    with safe_open(str(path), framework="pt") as f:
        meta = f.metadata() or {}
    arch = meta.get("arch") or ARCHS.get(name or "")
    m = {"yolov5nu": YOLOv5nu, "mobilenetv2": MobileNetV2}[arch]()
    m.load_state_dict(load_file(str(path)))
    return m.eval()


def _metadata(name: str, cfg, model_path: Path, seed: int) -> dict:
    from ..config import get_model_config

    spec = get_model_config(name)
    return {
        "name": name,
        "version": "1",
        "format": "safetensors",
        "arch": ARCHS[name],
        "platform": cfg.platform,
        "input": spec["input"],
        "output": spec["output"],
        "sha256": sha256_file(model_path),
        "bytes": model_path.stat().st_size,
        "weight_seed": seed,
        "created": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime()),
        "source": spec.get("source", ""),
    }


def build_repository(root: str | Path, *, models: list[str] | None = None, seed: int = 0, force: bool = False,
                     reference_compat: bool = False, pipeline: bool = True) -> dict:
    """Create/refresh a repository; existing files are kept unless ``force``."""
    root = Path(root)
    report = {}
    for name in models or list(ARCHS):
        d = root / name
        mp = d / "1" / MODEL_FILE
        actions = []
        if force or not mp.exists():
            export_model(name, mp, seed=seed)
            actions.append("model")
        cp = d / "config.pbtxt"
        cfg = mc.generate(name, reference_compat=reference_compat)
        if force or not cp.exists():
            cp.write_text(mc.dump(cfg, header=f"# {name}: generated from experiment.yaml"))
            actions.append("config")
        meta = d / "metadata.json"
        if force or not meta.exists() or actions:
            meta.write_text(json.dumps(_metadata(name, mc.parse(cp.read_text()), mp, seed), indent=2) + "\n")
            actions.append("metadata")
        report[name] = actions or ["present"]
    if pipeline:
        d = root / PIPELINE
        (d / "1").mkdir(parents=True, exist_ok=True)
        cp = d / "config.pbtxt"
        if force or not cp.exists():
            cp.write_text(mc.dump(mc.generate_pipeline(PIPELINE), header="# fused detect -> crop -> classify"))
            report[PIPELINE] = ["config"]
        else:
            report[PIPELINE] = ["present"]
    write_checksums(root)
    return report


def write_checksums(root: Path) -> Path:
    lines = [f"{sha256_file(p)}  {p.relative_to(root)}" for p in sorted(root.rglob(MODEL_FILE))]
    out = root / "checksums.txt"
    out.write_text("\n".join(lines) + ("\n" if lines else ""))
    return out


@dataclass
class ModelEntry:
    name: str
    path: Path
    config: object
    versions: list[int]
    metadata: dict

    def version_dir(self, version: int | None = None) -> Path:
        v = version if version is not None else self.versions[-1]
        return self.path / str(v)

    def model_file(self, version: int | None = None) -> Path:
        fn = self.config.default_model_filename or MODEL_FILE
        return self.version_dir(version) / fn


def _served_versions(cfg, found: list[int]) -> list[int]:
    vp = cfg.version_policy
    which = vp.WhichOneof("policy_choice") if cfg.HasField("version_policy") else None
    if which == "all":
        return found
    if which == "specific":
        return [v for v in found if v in set(vp.specific.versions)]
    n = vp.latest.num_versions if which == "latest" and vp.latest.num_versions else 1
    return found[-n:]


def scan_repository(root: str | Path) -> dict[str, ModelEntry]:
    """Model name -> entry for every directory with a config.pbtxt (Triton repository rules)."""
    root = Path(root)
    out = {}
    for d in sorted(p for p in root.iterdir() if p.is_dir()):
        cp = d / "config.pbtxt"
        if not cp.exists():
            continue
        cfg = mc.parse(cp.read_text())
        if not cfg.name:
            cfg.name = d.name
        found = sorted(int(v.name) for v in d.iterdir() if v.is_dir() and v.name.isdigit())
        meta = json.loads((d / "metadata.json").read_text()) if (d / "metadata.json").exists() else {}
        out[cfg.name] = ModelEntry(cfg.name, d, cfg, _served_versions(cfg, found), meta)
    return out


def verify_repository(root: str | Path) -> dict[str, list[str]]:
    """Problems per model (empty list = OK): config validity, files, sha256 vs metadata."""
    problems = {}
    for name, e in scan_repository(root).items():
        p = list(mc.validate(e.config))
        if e.config.platform != mc.ENSEMBLE:
            if not e.versions:
                p.append("no version directory")
            else:
                f = e.model_file()
                if not f.exists():
                    p.append(f"missing {f.relative_to(Path(root))}")
                elif e.metadata.get("sha256") and sha256_file(f) != e.metadata["sha256"]:
                    p.append("sha256 mismatch")
                elif not e.metadata:
                    p.append("missing metadata.json")
        else:
            known = scan_repository(root)
            for st in e.config.ensemble_scheduling.step:
                if st.model_name not in known:
                    p.append(f"ensemble step references unknown model '{st.model_name}'")
        problems[name] = p
    return problems


def sync_repository(src: str | Path, dst: str | Path, *, force: bool = False) -> list[str]:
    """Copy a repository (upload / init-container equivalent); returns copied relative paths."""
    src, dst = Path(src), Path(dst)
    copied = []
    for f in sorted(p for p in src.rglob("*") if p.is_file()):
        rel = f.relative_to(src)
        t = dst / rel
        if t.exists() and not force:
            continue
        t.parent.mkdir(parents=True, exist_ok=True)
        shutil.copy2(f, t)
        copied.append(str(rel))
    for d in sorted(p for p in src.rglob("*") if p.is_dir()):  # keep empty version dirs
        (dst / d.relative_to(src)).mkdir(parents=True, exist_ok=True)
    return copied


def init_flat(src: str | Path, dst: str | Path, models: list[str] | None = None) -> list[Path]:
    """Flat ``<dst>/<model>.safetensors`` files for the monolithic / microservices services."""
    entries = scan_repository(src)
    out = []
    Path(dst).mkdir(parents=True, exist_ok=True)
    for name in models or list(ARCHS):
        f = entries[name].model_file()
        t = Path(dst) / f"{name}.safetensors"
        shutil.copy2(f, t)
        out.append(t)
    return out
