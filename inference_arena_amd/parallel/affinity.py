"""Host-CPU placement of one serving rank per GPU.

The reference runs every service in a container limited to 2 vCPU (experiment.yaml:250-267); on an
MI355X node the host work per request (HTTP, multipart, JPEG decode, batching) is what scales with
the GPU count, so each rank gets its own CPU share next to its GPU:

* ``gpu_local_cpus(local_rank)`` reads the KFD topology in sysfs (no HIP call, so it is safe before
  any process is spawned or exec'd): the ``local_rank``-th GPU node, its PCI address and that
  device's ``local_cpulist`` (the CPUs of its NUMA node);
* ``rank_cpu_share(local_rank, local_world)`` splits those CPUs between the ranks whose GPUs sit on
  the same NUMA node, intersected with the CPUs this process may use; the decode workers pin
  themselves to that share (server/decode_pool.py ``cpus=``) and the rank process keeps the same set.

Everything degrades to "no pinning" (None) when the topology is unreadable (CPU-only hosts, containers
without /sys/class/kfd)."""
from __future__ import annotations

import os
from pathlib import Path

KFD_NODES = Path("/sys/class/kfd/kfd/topology/nodes")


def _parse_cpulist(text: str) -> list[int]:
    out: list[int] = []
    for part in text.strip().split(","):
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-")
            out.extend(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return out


def _props(node: Path) -> dict[str, int]:
    d: dict[str, int] = {}
    try:
        for line in (node / "properties").read_text().splitlines():
            k, _, v = line.partition(" ")
            try:
                d[k] = int(v)
            except ValueError:
                pass
    except OSError:
        pass
    return d


def gpu_nodes(root: Path = KFD_NODES) -> list[dict[str, int]]:
    """KFD GPU nodes (simd_count > 0) in node order, which is HIP's device order without HIP_VISIBLE_DEVICES."""
    if not root.is_dir():
        return []
    nodes = sorted((p for p in root.iterdir() if p.name.isdigit()), key=lambda p: int(p.name))
    return [pr for pr in (_props(n) for n in nodes) if pr.get("simd_count", 0) > 0]


def _pci_dir(props: dict[str, int], pci_root: Path = Path("/sys/bus/pci/devices")) -> Path | None:
    loc = props.get("location_id")
    if loc is None:
        return None
    bus, dev, fn = (loc >> 8) & 0xFF, (loc >> 3) & 0x1F, loc & 0x7
    p = pci_root / f"{props.get('domain', 0):04x}:{bus:02x}:{dev:02x}.{fn:x}"
    return p if p.exists() else None


def gpu_local_cpus(local_rank: int, root: Path = KFD_NODES, pci_root: Path = Path("/sys/bus/pci/devices")
                   ) -> tuple[list[int] | None, int]:
    """(CPUs of the NUMA node of GPU ``local_rank`` or None, that NUMA node id or -1)."""
    vis = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("ROCR_VISIBLE_DEVICES")
    nodes = gpu_nodes(root)
    idx = local_rank
    if vis:
        try:
            idx = [int(v) for v in vis.split(",")][local_rank]
        except (ValueError, IndexError):
            return None, -1
    if idx >= len(nodes):
        return None, -1
    d = _pci_dir(nodes[idx], pci_root)
    if d is None:
        return None, -1
    try:
        cpus = _parse_cpulist((d / "local_cpulist").read_text())
        numa = int((d / "numa_node").read_text().strip())
    except (OSError, ValueError):
        return None, -1
    return (cpus or None), numa


def rank_cpu_share(local_rank: int, local_world: int, root: Path = KFD_NODES,
                   pci_root: Path = Path("/sys/bus/pci/devices")) -> list[int] | None:
    """This rank's CPUs: its GPU's NUMA-local CPUs that this process may use, split evenly (contiguous
    blocks) between the ranks whose GPUs share that NUMA node.  None when unknown."""
    mine, numa = gpu_local_cpus(local_rank, root, pci_root)
    if not mine:
        return None
    allowed = set(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else set(mine)
    local = [c for c in mine if c in allowed]
    if not local:
        return None
    peers = [r for r in range(local_world) if gpu_local_cpus(r, root, pci_root)[1] == numa] or [local_rank]
    k, n = peers.index(local_rank) if local_rank in peers else 0, len(peers)
    per = max(1, len(local) // n)
    share = local[k * per:(k + 1) * per] if k < n - 1 else local[k * per:]
    return share or local


def cgroup_cpu_quota(path: Path = Path("/sys/fs/cgroup/cpu.max")) -> float | None:
    """The job's CPU quota in CPUs (cgroup v2 ``cpu.max``), None when unlimited or unreadable.  On the GPU pool
    the affinity mask shows the whole machine while this quota is the job's share.  ``ARENA_CPU_QUOTA``
    overrides it (tests of the N-rank sizing)."""
    env = os.environ.get("ARENA_CPU_QUOTA")
    if env:
        return float(env)
    try:
        quota, period = path.read_text().split()[:2]
        if quota != "max":
            return max(1.0, int(quota) / int(period))
    except (OSError, ValueError):
        pass
    return None


def usable_cpus_per_rank(share: list[int] | None, local_world: int) -> int:
    """CPUs one rank may really use: its pinned share (or the affinity mask), capped by the job's cgroup quota
    divided between the node's ranks — every rank sees the whole quota, so sizing per rank from it alone would
    oversubscribe the job ``local_world`` times."""
    n = len(share) if share else (len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity")
                                  else (os.cpu_count() or 8))
    q = cgroup_cpu_quota()
    if q is not None:
        n = min(n, max(1, int(q // max(1, local_world))))
    return max(1, n)


def host_thread_plan(usable: int) -> dict[str, int]:
    """Host threads of one serving rank for ``usable`` CPUs: HTTP epoll threads, native split-decoder threads
    (marker parse + Huffman decode, ~0.2 ms per COCO-sized q90 JPEG on the GPU box), load-generator threads of
    the bench, PIL processes (only uploads the split decoder does not cover).  The batcher / executor threads
    come on top: one each per instance."""
    io = 4 if usable >= 12 else max(1, usable // 4)
    decode = max(1, min(12, usable // 2))
    return {"http_io": io, "decode_threads": decode, "loadgen": 2 if usable >= 8 else 1, "pil_procs": 1}


def pin(cpus: list[int] | None) -> bool:
    """Restrict the calling process (and the threads it creates afterwards) to ``cpus``."""
    if not cpus or not hasattr(os, "sched_setaffinity"):
        return False
    try:
        os.sched_setaffinity(0, cpus)
        return True
    except OSError:
        return False


def rank_host_setup(gpu_rank: int, local_world: int, *, do_pin: bool = True) -> dict:
    """One serving process per GPU: its CPU share (the GPU's NUMA-local CPUs split between the node's ranks on
    that NUMA node), the CPUs it may really use (capped by the job's cgroup quota divided by ``local_world``), and
    the host thread plan for that many CPUs; pins the process to the share.  Every process of the Triton arm's
    per-GPU layout (model servers, gateways) and the monolithic replicas size themselves with it, so the host
    plan scales with the GPU count.  ``ARENA_HTTP_THREADS`` / ``ARENA_DECODE_THREADS``
    still override the plan."""
    share = rank_cpu_share(gpu_rank, max(1, local_world))
    usable = usable_cpus_per_rank(share, max(1, local_world))
    plan = host_thread_plan(usable)
    if os.environ.get("ARENA_HTTP_THREADS"):
        plan["http_io"] = int(os.environ["ARENA_HTTP_THREADS"])
    if os.environ.get("ARENA_DECODE_THREADS"):
        plan["decode_threads"] = int(os.environ["ARENA_DECODE_THREADS"])
    pinned = pin(share) if do_pin else False
    return {"gpu": int(gpu_rank), "local_world": int(local_world), "cpus": share, "usable_cpus": usable,
            "pinned": pinned, "plan": plan}


def rank_info_metrics(info: dict, arch: str) -> str:
    """Prometheus text of a rank's host placement: ``arena_rank_usable_cpus`` and ``arena_rank_threads``."""
    cpus = info.get("cpus")
    cl = ",".join(str(c) for c in cpus) if cpus else "all"
    g = info.get("gpu", 0)
    lines = ["# HELP arena_rank_usable_cpus CPUs this serving process may use (its share of the node)",
             "# TYPE arena_rank_usable_cpus gauge",
             f'arena_rank_usable_cpus{{arch="{arch}",gpu="{g}",cpus="{cl}"}} {info.get("usable_cpus", 0)}',
             "# HELP arena_rank_threads host threads of this serving process by role",
             "# TYPE arena_rank_threads gauge"]
    for role, n in sorted((info.get("plan") or {}).items()):
        lines.append(f'arena_rank_threads{{arch="{arch}",gpu="{g}",role="{role}"}} {n}')
    return "\n".join(lines) + "\n"
