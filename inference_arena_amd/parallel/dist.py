"""Process-group helpers for one-process-per-GPU replicas.

The reference scales only by container count and has no collectives
(SURVEY.md §2.4).  Here every GPU replica is its own process; at start-up the
replicas join one ``torch.distributed`` group — backend ``nccl``, which is
RCCL over xGMI on MI355X (``gloo`` on CPU for tests) — and rank 0's folded
weight blob is broadcast to all replicas in one collective, so every replica
serves bit-identical weights without each one re-reading the model
repository.  Per-replica statistics are all-reduced / all-gathered at the
end of a benchmark.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import numpy as np
import torch
import torch.distributed as dist


@dataclass
class DistInfo:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    backend: str = "none"

    @property
    def is_main(self) -> bool:
        return self.rank == 0


def init_from_env(backend: str | None = None) -> DistInfo:
    """Join the process group described by torchrun's env vars (no-op for world 1)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    if world <= 1:
        return DistInfo(0, 1, local, "none")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if backend == "nccl":
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", local))
    else:
        dist.init_process_group(backend, rank=rank, world_size=world)
    return DistInfo(rank, world, local, backend)


def _dev(info: DistInfo) -> torch.device:
    return torch.device("cuda", info.local_rank) if info.backend == "nccl" else torch.device("cpu")


def broadcast_blob(blob: np.ndarray | None, info: DistInfo, src: int = 0) -> np.ndarray:
    """Broadcast a uint8 blob from ``src`` to every rank (one RCCL broadcast over xGMI)."""
    if info.world <= 1:
        assert blob is not None
        return blob
    dev = _dev(info)
    n = torch.tensor([blob.nbytes if blob is not None and info.rank == src else 0], dtype=torch.int64, device=dev)
    dist.broadcast(n, src)
    if info.rank == src:
        t = torch.from_numpy(np.ascontiguousarray(blob)).to(dev)
    else:
        t = torch.empty(int(n.item()), dtype=torch.uint8, device=dev)
    dist.broadcast(t, src)
    return t.cpu().numpy()


def broadcast_blob_device(blob: np.ndarray | None, info: DistInfo, src: int = 0) -> torch.Tensor:
    """As ``broadcast_blob`` but the result stays on this rank's GPU (RCCL over xGMI lands it there): hand it
    to ``Executor.set_weights_device`` (device-to-device copy, no host round trip)."""
    dev = _dev(info)
    if info.world <= 1:
        assert blob is not None
        return torch.from_numpy(np.ascontiguousarray(blob)).to(dev)
    n = torch.tensor([blob.nbytes if blob is not None and info.rank == src else 0], dtype=torch.int64, device=dev)
    dist.broadcast(n, src)
    if info.rank == src:
        t = torch.from_numpy(np.ascontiguousarray(blob)).to(dev)
    else:
        t = torch.empty(int(n.item()), dtype=torch.uint8, device=dev)
    dist.broadcast(t, src)
    return t


def broadcast_object(obj, info: DistInfo, src: int = 0):
    if info.world <= 1:
        return obj
    lst = [obj if info.rank == src else None]
    dist.broadcast_object_list(lst, src, device=_dev(info) if info.backend == "nccl" else None)
    return lst[0]


def allreduce_max(v: float, info: DistInfo) -> float:
    if info.world <= 1:
        return float(v)
    t = torch.tensor([float(v)], dtype=torch.float64, device=_dev(info))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def allgather_floats(vals: list[float], info: DistInfo) -> list[list[float]]:
    if info.world <= 1:
        return [list(vals)]
    out: list = [None] * info.world
    dist.all_gather_object(out, list(vals))
    return out


def allgather_objects(obj, info: DistInfo) -> list:
    """Every rank's ``obj`` (picklable), in rank order."""
    if info.world <= 1:
        return [obj]
    out: list = [None] * info.world
    dist.all_gather_object(out, obj)
    return out


def barrier(info: DistInfo) -> None:
    if info.world > 1:
        if info.backend == "nccl":
            dist.barrier(device_ids=[info.local_rank])
        else:
            dist.barrier()


def shutdown(info: DistInfo) -> None:
    if info.world > 1 and dist.is_initialized():
        dist.destroy_process_group()


def device_identity(dev: int | None, rank: int, fake: bool = False) -> dict:
    """The physical GPU a rank drives: PCI domain:bus:device plus the HIP UUID when torch reports them.  The
    scaling record (bench.py ``rank_devices``) carries one per rank, so an N-GPU result can be checked to come
    from N distinct devices, not N ranks sharing one (``world_size_checked`` alone cannot show that).  ``fake``:
    the CPU fake engine, one synthetic id per rank (``ARENA_TEST_DUP_BUS=1``: all ranks the same id, the
    duplicate check's own test)."""
    if fake or dev is None:
        bus = "fake:00" if os.environ.get("ARENA_TEST_DUP_BUS") == "1" else f"fake:{rank:02d}"
        return {"rank": rank, "device": dev, "pci_bus_id": bus, "uuid": None, "name": "fake-engine"}
    import torch

    p = torch.cuda.get_device_properties(dev)
    bus = "%04x:%02x:%02x.0" % (int(getattr(p, "pci_domain_id", 0)), int(getattr(p, "pci_bus_id", 0)),
                                int(getattr(p, "pci_device_id", 0)))
    uuid = str(getattr(p, "uuid", "")) or None
    return {"rank": rank, "device": int(dev), "pci_bus_id": bus, "uuid": uuid, "name": p.name}


def check_distinct_devices(ids: list[dict], shared_ok: bool) -> None:
    """Refuse a multi-rank result in which two ranks drove the same physical GPU, unless that is the explicit
    rehearsal mode (``ARENA_SHARED_GPU=1``: every rank on device 0 of a one-GPU box)."""
    seen: dict[str, int] = {}
    for d in ids:
        key = d.get("pci_bus_id")
        if key in seen and not shared_ok:
            raise RuntimeError(f"ranks {seen[key]} and {d.get('rank')} drive the same GPU ({key}); a scaling "
                               f"result needs one device per rank (set ARENA_SHARED_GPU=1 only for a rehearsal)")
        seen.setdefault(key, d.get("rank"))
