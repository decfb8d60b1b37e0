"""RQ2 (resource efficiency, cost per request) and RQ3 (operational complexity) for the three arms.

The reference declares these metrics (/root/reference/experiment.yaml:47-60: ``cpu_utilization_percent``,
``memory_usage_mb``, ``cost_per_1000_requests_usd``, ``application_code_loc``, ``configuration_loc``,
``deployment_time``) but ships no code computing them (its ``analysis/`` holds only ``.gitkeep``).  Here:

* cost per 1000 requests = (GPU-hours x price + vCPU-hours x price) per second / throughput x 1000, with the
  prices an explicit, configurable assumption (``cost`` section of experiment.yaml), not market data;
* application / configuration LOC per arm, counted over the modules and files that make up that arm in this
  repository (non-blank, non-comment lines);
* the RQ2 columns measured by loadgen/resources.py during each load level are carried through.
"""
from __future__ import annotations

from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]

# modules / files per arm (shared engine + kernels count for every arm and are reported separately)
ARM_CODE = {
    "monolithic": ["inference_arena_amd/server/monolithic.py", "inference_arena_amd/server/backends.py",
                   "inference_arena_amd/server/app_common.py", "inference_arena_amd/server/schemas.py",
                   "inference_arena_amd/server/replica.py", "inference_arena_amd/server/batching.py",
                   "csrc/runtime/http_front.cpp", "csrc/runtime/http_front.h"],
    "microservices": ["inference_arena_amd/server/detection_service.py",
                      "inference_arena_amd/server/classification_service.py",
                      "inference_arena_amd/server/grpc_client.py", "inference_arena_amd/server/crop_codec.py",
                      "inference_arena_amd/server/service_backends.py", "inference_arena_amd/server/schemas.py",
                      "inference_arena_amd/server/app_common.py", "inference_arena_amd/proto/inference_api.py",
                      "inference_arena_amd/proto/builder.py"],
    "triton": ["inference_arena_amd/server/model_server.py", "inference_arena_amd/server/modelserver_core.py",
               "inference_arena_amd/server/gateway.py", "inference_arena_amd/server/kserve_client.py",
               "inference_arena_amd/server/schemas.py", "inference_arena_amd/repository/model_config.py",
               "inference_arena_amd/repository/store.py", "inference_arena_amd/proto/builder.py"],
}
ARM_CONFIG = {
    "monolithic": ["deploy/compose/monolithic.yml", "deploy/Dockerfile"],
    "microservices": ["deploy/compose/microservices.yml", "deploy/Dockerfile"],
    "triton": ["deploy/compose/triton.yml", "deploy/Dockerfile"],
}
SHARED_CODE_DIRS = ["inference_arena_amd/engine", "inference_arena_amd/ops", "csrc/kernels", "csrc/runtime"]


def count_loc(path: Path) -> int:
    """Non-blank lines that are not comments: ``#`` lines in Python / YAML / Dockerfiles, ``//`` lines and
    ``/* ... */`` blocks in C++ / HIP."""
    c_like = path.suffix in (".cpp", ".h", ".hip", ".cu")
    n, in_block = 0, False
    for raw in path.read_text(errors="replace").splitlines():
        line = raw.strip()
        if not line:
            continue
        if c_like:
            if in_block:
                in_block = "*/" not in line
                continue
            if line.startswith("/*"):
                in_block = "*/" not in line
                continue
            if line.startswith("//"):
                continue
        elif line.startswith("#"):
            continue
        n += 1
    return n


def complexity_report(root: Path = ROOT) -> dict:
    """RQ3: application / configuration LOC per arm (+ the shared engine that every arm uses)."""
    out = {}
    for arm, files in ARM_CODE.items():
        app = sum(count_loc(root / f) for f in files if (root / f).exists())
        cfg = sum(count_loc(root / f) for f in ARM_CONFIG[arm] if (root / f).exists())
        out[arm] = {"application_code_loc": app, "configuration_loc": cfg,
                    "files": [f for f in files + ARM_CONFIG[arm] if (root / f).exists()]}
    shared = 0
    for d in SHARED_CODE_DIRS:
        for f in sorted((root / d).rglob("*")):
            if f.suffix in (".py", ".cpp", ".h", ".hip") and f.is_file():
                shared += count_loc(f)
    out["shared_engine_loc"] = shared
    return out


def cost_per_1000_requests(throughput_rps: float, *, gpus: int, gpu_hour_usd: float, vcpus: float = 0.0,
                           vcpu_hour_usd: float = 0.0) -> float:
    """USD per 1000 requests at a sustained ``throughput_rps`` on ``gpus`` GPUs and ``vcpus`` host cores."""
    if not throughput_rps or throughput_rps <= 0:
        return float("nan")
    per_s = (gpus * gpu_hour_usd + vcpus * vcpu_hour_usd) / 3600.0
    return per_s / throughput_rps * 1000.0


def enrich_sweep_rows(rows: list[dict], *, gpus: int, cost: dict) -> list[dict]:
    """Add ``cost_per_1000_requests_usd`` to loadgen sweep rows; host vCPUs billed as the measured CPU use
    (``cpu_utilization_percent`` / 100) when the row has it, else the arm's configured container vCPUs."""
    out = []
    for r in rows:
        r = dict(r)
        cpu = r.get("cpu_utilization_percent")
        vcpus = (float(cpu) / 100.0) if cpu == cpu and cpu is not None else float(cost.get("vcpus", 0.0))
        r["cost_per_1000_requests_usd"] = cost_per_1000_requests(
            float(r.get("throughput_rps", 0.0)), gpus=gpus, gpu_hour_usd=float(cost.get("gpu_hour_usd", 0.0)),
            vcpus=vcpus, vcpu_hour_usd=float(cost.get("vcpu_hour_usd", 0.0)))
        out.append(r)
    return out
