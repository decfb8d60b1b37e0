"""Thread-safe lazy registry of compiled GPU models (the ORT-session registry's role).

Reference: src/shared/model/registry.py:88-343 — ``ModelRegistry`` caches one
ONNX Runtime session per model behind a lock, with a ``SessionConfig``
(threads, providers), ``get_session``, ``get_model_info``, ``is_loaded``,
``preload_all``, ``clear_cache``, ``list_available`` and a process-wide
default registry.  Here a "session" is a ``GpuProgramRunner`` (executor +
captured hipGraphs) built from a model repository entry or the seeded
default weights; ``SessionConfig`` holds the device, batch buckets and
executor settings instead of ORT thread counts.
"""
from __future__ import annotations

import threading
from dataclasses import dataclass, field
from pathlib import Path


@dataclass
class SessionConfig:
    device: int = 0
    buckets: list[int] = field(default_factory=lambda: [1, 2, 4, 8, 16, 32])
    host_threads: int | None = None
    crop_cap_per_image: int | None = None
    weight_seed: int = 0


@dataclass
class ModelInfo:
    name: str
    kind: str
    input_shape: tuple
    output_shape: tuple
    weights_bytes: int
    arena_bytes: dict
    source: str


MODEL_KINDS = ("yolov5n", "mobilenetv2", "pipeline", "detector", "classifier", "frame_classifier", "split")


def build_session(kind: str, yolo=None, mnet=None, *, device: int = 0, buckets=None, dtype: str | None = None,
                  **kw):
    """The one construction point of a compiled GPU model (every server backend and the registry use it).

    kind: ``yolov5n`` / ``mobilenetv2`` (raw tensor models, the model server's per-model entries),
    ``pipeline`` (fused detector -> crops -> classifier), ``detector`` / ``classifier`` (the microservices
    halves), ``frame_classifier`` (crop gather + classifier over device-resident frames: arm B device
    transport) or ``split`` (pipeline with detection on ``device`` and classification on ``cls_device``).
    Extra keywords go to the engine class (weights, host_threads, crop_cap_per_image, cls_device)."""
    from .pipeline import GpuClassifier, GpuDetector, GpuFrameClassifier, GpuPipeline, GpuTensorModel, SplitPipeline

    common = dict(buckets=buckets, dtype=dtype)
    if kind == "yolov5n":
        return GpuTensorModel.yolo(yolo, device=device, **common)
    if kind == "mobilenetv2":
        return GpuTensorModel.mobilenet(mnet, device=device, **common)
    if kind == "pipeline":
        return GpuPipeline(yolo, mnet, device=device, **common, **kw)
    if kind == "detector":
        return GpuDetector(yolo, device=device, **common)
    if kind == "classifier":
        return GpuClassifier(mnet, device=device, **common)
    if kind == "frame_classifier":
        return GpuFrameClassifier(mnet, device=device, **common, **kw)
    if kind == "split":
        return SplitPipeline(yolo, mnet, det_device=device, cls_device=int(kw.pop("cls_device", 1)), **common, **kw)
    raise KeyError(f"unknown model '{kind}' (available: {', '.join(MODEL_KINDS)})")


class ModelRegistry:
    def __init__(self, models_dir: str | Path | None = None, config: SessionConfig | None = None):
        self.models_dir = Path(models_dir) if models_dir else None
        self.config = config or SessionConfig()
        self._lock = threading.Lock()
        self._sessions: dict = {}

    def list_available(self) -> list[str]:
        return list(MODEL_KINDS)

    def _modules(self):
        from ..models.zoo import resolve_models

        return resolve_models(str(self.models_dir) if self.models_dir else None, self.config.weight_seed)

    def _build(self, name: str):
        yolo, mnet = self._modules()
        c = self.config
        kw = {}
        if name == "pipeline":
            kw = dict(host_threads=c.host_threads, crop_cap_per_image=c.crop_cap_per_image)
        return build_session(name, yolo, mnet, device=c.device, buckets=c.buckets, **kw)

    def get_session(self, name: str):
        with self._lock:
            s = self._sessions.get(name)
            if s is None:
                s = self._build(name)
                self._sessions[name] = s
            return s

    def get_model_info(self, name: str) -> ModelInfo:
        s = self.get_session(name)
        meta = s.program.meta
        ins = getattr(s, "input_shape", ("H", "W", 3))
        outs = getattr(s, "output_shape", ("detections", "top5"))
        return ModelInfo(name, str(meta.get("kind", name)), tuple(ins), tuple(outs), int(s.program.weights.nbytes),
                         dict(s.arena_bytes), str(self.models_dir or f"seed {self.config.weight_seed}"))

    def is_loaded(self, name: str) -> bool:
        with self._lock:
            return name in self._sessions

    def preload_all(self, names: list[str] | None = None) -> None:
        for n in names or ["pipeline"]:
            self.get_session(n)

    def clear_cache(self) -> None:
        with self._lock:
            self._sessions.clear()


_default: ModelRegistry | None = None
_default_lock = threading.Lock()


def get_default_registry(models_dir: str | Path | None = None, config: SessionConfig | None = None) -> ModelRegistry:
    global _default
    with _default_lock:
        if _default is None:
            _default = ModelRegistry(models_dir, config)
        return _default


def reset_default_registry() -> None:
    global _default
    with _default_lock:
        _default = None
