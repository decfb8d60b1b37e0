"""Model-instance placement over the GPUs of one node.

Triton's ``instance_group [{count: c, kind: KIND_GPU, gpus: [g0, g1, ...]}]``
places ``c`` instances of the model on EACH listed GPU (no ``gpus`` = every
visible GPU); the reference declares one KIND_CPU instance
(reference infrastructure/minio/triton_config.py:72-74,114-117).  The same
rule drives the model server (server/modelserver_core.py), the microservices
backends (``ARENA_GPUS``) and the launcher (scripts/start_arena.py), so an
N-GPU deployment is data-parallel in every arm.
"""
from __future__ import annotations

import os


def visible_gpus() -> int:
    """Number of GPUs this process may use, without initialising the GPU (torch.cuda.device_count on this
    image does not create a context)."""
    env = os.environ.get("ARENA_VISIBLE_GPUS")
    if env:
        return max(1, int(env))
    try:
        import torch

        return max(1, torch.cuda.device_count())
    except Exception:  # noqa: BLE001 - no torch / no GPU: one logical device
        return 1


def parse_gpu_list(spec: str | int | list | None, default: int = 0) -> list[int]:
    """``"0,1,3"`` / ``"0-3"`` / ``2`` / ``[0, 1]`` -> sorted unique GPU ids (``default`` when empty)."""
    if spec is None or spec == "" or spec == []:
        return [int(default)]
    if isinstance(spec, int):
        return [spec]
    if isinstance(spec, (list, tuple)):
        return sorted({int(g) for g in spec})
    out: set[int] = set()
    for part in str(spec).split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-", 1)
            out.update(range(int(a), int(b) + 1))
        else:
            out.add(int(part))
    if not out:
        return [int(default)]
    return sorted(out)


def instance_devices(groups, *, default_gpu: int = 0, n_visible: int | None = None) -> list[int]:
    """Device of every model instance for a list of instance groups.

    ``groups``: objects or dicts with ``count``, ``kind`` and ``gpus``.  KIND_GPU (or AUTO) groups give
    ``count`` instances per listed GPU, every visible GPU when ``gpus`` is empty; KIND_CPU groups still
    serve from ``default_gpu`` in the GPU server (the reference's CPU instance maps onto the device).
    """
    n_visible = visible_gpus() if n_visible is None else int(n_visible)
    devs: list[int] = []

    def field(g, k, d):
        return g.get(k, d) if isinstance(g, dict) else getattr(g, k, d)

    for g in groups or []:
        count = max(0, int(field(g, "count", 1) or 0))
        if count == 0:
            continue
        kind = field(g, "kind", "KIND_GPU")
        kind = kind if isinstance(kind, str) else {0: "KIND_AUTO", 1: "KIND_GPU", 2: "KIND_CPU"}.get(int(kind), "")
        gpus = [int(x) for x in (field(g, "gpus", []) or [])]
        if kind == "KIND_CPU":
            gpus = [default_gpu]
        elif not gpus:
            gpus = list(range(n_visible))
        for x in gpus:
            if x < 0 or x >= n_visible:
                raise ValueError(f"instance_group lists GPU {x}, but only {n_visible} visible")
        for x in gpus:
            devs += [x] * count
    return devs or [int(default_gpu)]


def endpoints(spec: str) -> list[str]:
    """Comma-separated gRPC endpoints (``host:port,host:port``)."""
    return [e.strip() for e in str(spec).split(",") if e.strip()]
