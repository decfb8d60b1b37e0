"""Environment-driven service settings (pydantic-settings replacement).

The reference configures each service with pydantic-settings classes
(architectures/*/app/config.py: LOG_LEVEL, PORT, MODELS_DIR,
CLASSIFICATION_GRPC_ENDPOINT, LABELS_FILE, TRITON_GRPC_ENDPOINT,
TRITON_TIMEOUT_SECONDS; case-sensitive names, optional .env file).
pydantic-settings is not installed here, so ``Settings`` reads the same
variables from the environment and an optional ``.env`` file itself and
validates them with pydantic.
"""
from __future__ import annotations

import functools
import os
from pathlib import Path

from pydantic import BaseModel


def _read_dotenv(path: Path) -> dict[str, str]:
    out: dict[str, str] = {}
    if not path.exists():
        return out
    for line in path.read_text(encoding="utf-8").splitlines():
        line = line.strip()
        if not line or line.startswith("#") or "=" not in line:
            continue
        k, v = line.split("=", 1)
        v = v.strip()
        if v[:1] in ("'", '"') and v[0] in v[1:]:
            v = v[1:v.index(v[0], 1)]  # quoted value: keep '#' inside the quotes
        else:
            v = v.split(" #", 1)[0].split("\t#", 1)[0].strip()  # unquoted: drop an inline comment
        out[k.strip()] = v
    return out


class Settings(BaseModel):
    LOG_LEVEL: str = "INFO"
    PORT: int = 8100
    HOST: str = "0.0.0.0"
    MODELS_DIR: str = "model_repository"
    LABELS_FILE: str = ""
    CLASSIFICATION_GRPC_ENDPOINT: str = "127.0.0.1:8201"
    TRITON_GRPC_ENDPOINT: str = "127.0.0.1:8001"
    TRITON_HTTP_ENDPOINT: str = "127.0.0.1:8000"
    TRITON_TIMEOUT_SECONDS: float = 60.0
    # arena additions
    ARENA_DEVICE: str = "gpu"          # gpu | cpu | fake (host-only EchoInstance: CPU tests of node layouts)
    ARENA_GPU: int = 0
    ARENA_GPUS: str = ""               # GPUs one process drives ("0,1" / "0-7"); '' = ARENA_GPU only
    ARENA_CLS_GPU: int = -1            # split topology: classification GPU (crops handed over device to device)
    ARENA_MAX_BATCH: int = 32
    ARENA_QUEUE_DELAY_US: int = 500
    ARENA_DECODE_THREADS: int = 8
    ARENA_CONFIDENCE: str = ""          # logit | softmax ('' = topology default)
    ARENA_CROP_TRANSPORT: str = "jpeg"  # jpeg (reference) | png | raw | device (IPC frame hand-off)
    ARENA_DEVICE_RING_SLOTS: int = 512  # device transport: frames in flight per detection process
    ARENA_FANOUT: str = "parallel"      # parallel (one Classify per crop, reference) | batch (one ClassifyBatch)
    ARENA_GATEWAY_MODE: str = "pipeline"  # pipeline (one fused ensemble RPC) | tensor (reference per-model RPCs)
    ARENA_INSTANCES: int = 1            # executor instances per GPU behind one batcher
    ARENA_WEIGHT_SEED: int = 0
    ARENA_FAULT_EVERY: int = 0          # inject a failure every k-th request (0 = off)
    ARENA_INFER_SERVICE: int = 0        # classification gRPC server also serves inference.InferenceService/Infer

    @classmethod
    def from_env(cls, env_file: str | Path = ".env", **overrides) -> "Settings":
        vals: dict[str, str] = _read_dotenv(Path(env_file))
        for k in cls.model_fields:
            if k in os.environ:
                vals[k] = os.environ[k]
        vals.update({k: v for k, v in overrides.items() if v is not None})
        return cls(**vals)


@functools.lru_cache
def get_settings() -> Settings:
    return Settings.from_env()
