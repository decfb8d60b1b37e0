"""Resource sampling during a load level (experiment.yaml RQ2: ``cpu_utilization_percent``,
``memory_usage_mb``; reference: /root/reference/experiment.yaml:47-53 — the reference collects these from
cAdvisor through Prometheus, infrastructure/prometheus/prometheus.yml:17-20, and has no in-process sampler).

``ResourceSampler`` follows the arm's server processes — given as PIDs, or discovered as the processes listening
on the arm's ports (``gpu.ports`` in experiment.yaml) — and all their children (decode workers, replicas), and
samples every ``interval`` seconds: summed CPU % (100 = one core), summed resident memory, and, when the MI355X
telemetry reader (metrics/gpu.py) finds a device, GPU busy % and VRAM.
"""
from __future__ import annotations

import os
import re
import threading
import time

import numpy as np


def pids_listening_on(ports: list[int]) -> list[int]:
    """PIDs of the processes holding a listening TCP socket on any of ``ports`` (best effort)."""
    import psutil

    out = set()
    try:
        conns = psutil.net_connections(kind="tcp")
    except (psutil.AccessDenied, PermissionError):
        conns = []
    for c in conns:
        if c.status == psutil.CONN_LISTEN and c.laddr and c.laddr.port in ports and c.pid:
            out.add(c.pid)
    return sorted(out)


class ResourceSampler:
    def __init__(self, pids: list[int], interval: float = 1.0, gpu: bool = True) -> None:
        import psutil

        self.interval = interval
        self.roots = [psutil.Process(p) for p in pids if psutil.pid_exists(p)]
        self.samples: list[tuple[float, float, float, float | None, float | None]] = []
        self.by_role: dict[str, list[float]] = {}  # CPU % per process role, summed over that role's processes
        self.mem_by_role: dict[str, list[float]] = {}  # RSS MB per process role (which service grows)
        self._stop = threading.Event()
        self._thread: threading.Thread | None = None
        self._cache: dict = {}
        # CPU % per (role, thread class): the native threads name themselves (arena-http-io, arena-jpeg,
        # arena-batcher, ...); HIP runtime and Python threads keep the process name
        self.by_thread: dict[tuple[str, str], list[float]] = {}
        self._ticks: dict[tuple[int, int], tuple[str, int]] = {}
        self._t_prev: float | None = None
        self._hz = os.sysconf("SC_CLK_TCK") if hasattr(os, "sysconf") else 100
        self._gpu = None
        if gpu:
            try:
                from ..metrics.gpu import GpuTelemetry

                t = GpuTelemetry()
                # amdsmi / amd-smi only: the torch fallback would initialise a GPU context in the load generator
                self._gpu = t if t.source in ("amdsmi", "cli") else None
            except Exception:  # noqa: BLE001 - no device / reader: CPU-side metrics only
                self._gpu = None

    def _procs(self):
        """The process trees, as the same psutil.Process objects from sample to sample: cpu_percent(None) measures
        since the previous call on that object, so a fresh object per sample would always read 0."""
        import psutil

        live = {}
        for r in self.roots:
            try:
                for p in [r] + r.children(recursive=True):
                    live[p.pid] = self._cache.get(p.pid, p)
            except psutil.NoSuchProcess:
                continue
        for pid, p in live.items():
            if pid not in self._cache:
                self._cache[pid] = p
                try:
                    p.cpu_percent(None)  # prime: its first real reading comes at the next sample
                except psutil.NoSuchProcess:
                    pass
        return list(live.values())

    def _sample(self, procs) -> None:
        import psutil

        cpu = mem = 0.0
        roles: dict[str, float] = {}
        role_mem: dict[str, float] = {}
        for p in procs:
            try:
                c = p.cpu_percent(None)
                m = p.memory_info().rss / 2 ** 20
                cpu += c
                mem += m
                r = self._role(p)
                roles[r] = roles.get(r, 0.0) + c
                role_mem[r] = role_mem.get(r, 0.0) + m
            except psutil.NoSuchProcess:
                continue
        for r, c in roles.items():
            self.by_role.setdefault(r, []).append(c)
        for r, m in role_mem.items():
            self.mem_by_role.setdefault(r, []).append(m)
        self._sample_threads(procs)
        busy = vram = None
        if self._gpu is not None:
            try:
                rows = self._gpu.sample()
                util = [r["util"] for r in rows if "util" in r]
                mems = [r["mem"] for r in rows if "mem" in r]
                busy = float(np.mean(util)) if util else None
                vram = float(np.sum(mems)) / 2 ** 20 if mems else None
            except Exception:  # noqa: BLE001
                pass
        self.samples.append((time.time(), cpu, mem, busy, vram))

    @staticmethod
    def thread_class(comm: str) -> str:
        """Thread name -> class: trailing digits / separators dropped (arena-jpeg3 -> arena-jpeg)."""
        return re.sub(r"[-_:.]?\d+$", "", comm.strip()) or comm

    def _sample_threads(self, procs) -> None:
        """Per-thread utime + stime from /proc/<pid>/task/*/stat since the previous sample, summed by (role,
        thread class) as CPU % (Linux only; best effort)."""
        now = time.monotonic()
        dt = None if self._t_prev is None else now - self._t_prev
        self._t_prev = now
        acc: dict[tuple[str, str], float] = {}
        for p in procs:
            role = self._cache.get(("role", p.pid)) or "other"
            base = f"/proc/{p.pid}/task"
            try:
                tids = os.listdir(base)
            except OSError:
                continue
            for tid in tids:
                try:
                    with open(f"{base}/{tid}/stat") as f:
                        st = f.read()
                except OSError:
                    continue
                l, r = st.find("("), st.rfind(")")
                if l < 0 or r < 0:
                    continue
                fields = st[r + 2:].split()
                try:
                    ticks = int(fields[11]) + int(fields[12])  # utime, stime (fields 14, 15 of stat)
                except (IndexError, ValueError):
                    continue
                key = (p.pid, int(tid))
                cls = self.thread_class(st[l + 1:r])
                prev = self._ticks.get(key)
                self._ticks[key] = (cls, ticks)
                if dt and prev is not None:
                    acc[(role, cls)] = acc.get((role, cls), 0.0) + 100.0 * (ticks - prev[1]) / self._hz / dt
        if dt:
            for k, v in acc.items():
                self.by_thread.setdefault(k, []).append(v)

    def _role(self, p) -> str:
        """Process role from the command line: the arm's services (``--arch X`` of the replica launcher, the model
        server, the classification service), the decode workers (forked from the multiprocessing fork server),
        and for spawned children (replicas) the role of the parent."""
        key = ("role", p.pid)
        role = self._cache.get(key)
        if role is not None:
            return role
        try:
            args = p.cmdline()
        except Exception:  # noqa: BLE001 - vanished / no access
            args = []
        cmd = " ".join(args)
        role = "other"
        if "forkserver" in cmd:
            role = "decode_workers"
        elif "--arch" in args and args.index("--arch") + 1 < len(args):
            role = args[args.index("--arch") + 1]
        elif "model_server" in cmd:
            role = "model_server"
        elif "classification_service" in cmd:
            role = "classification"
        elif "native_front" in cmd:
            role = "monolithic"
        elif "spawn_main" in cmd or "multiprocessing" in cmd:
            try:
                parent = p.parent()
                role = self._role(parent) if parent is not None else "other"
            except Exception:  # noqa: BLE001
                role = "other"
        self._cache[key] = role
        return role

    def _run(self) -> None:
        self._procs()  # prime every process's cpu counter
        while not self._stop.wait(self.interval):
            procs = self._procs()
            self._sample(procs)

    def start(self) -> "ResourceSampler":
        self._thread = threading.Thread(target=self._run, daemon=True)
        self._thread.start()
        return self

    def stop(self) -> dict:
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=5 * self.interval + 1)
        return self.summary()

    def summary(self) -> dict:
        if not self.samples:
            return {"cpu_utilization_percent": float("nan"), "memory_usage_mb": float("nan"), "resource_samples": 0}
        a = np.asarray([s[1:3] for s in self.samples], dtype=np.float64)
        out = {
            "cpu_utilization_percent": float(a[:, 0].mean()),   # 100 = one core busy
            "cpu_utilization_percent_max": float(a[:, 0].max()),
            "memory_usage_mb": float(a[:, 1].mean()),
            "memory_usage_mb_max": float(a[:, 1].max()),
            "resource_samples": len(self.samples),
        }
        out["cpu_percent_by_role"] = {r: round(float(np.mean(v)), 1) for r, v in sorted(self.by_role.items())}
        # RSS per role, mean and last sample: run-to-run growth can be pinned to one service
        out["memory_mb_by_role"] = {r: {"mean": round(float(np.mean(v)), 1), "last": round(float(v[-1]), 1)}
                                    for r, v in sorted(self.mem_by_role.items())}
        if self.by_thread:
            n = max(len(v) for v in self.by_thread.values())
            by: dict[str, dict[str, float]] = {}
            for (role, cls), v in sorted(self.by_thread.items()):
                pct = float(np.sum(v)) / n  # a class absent from some samples counted 0 there
                if pct >= 0.5:
                    by.setdefault(role, {})[cls] = round(pct, 1)
            out["cpu_percent_by_thread"] = by
        busy = [s[3] for s in self.samples if s[3] is not None]
        vram = [s[4] for s in self.samples if s[4] is not None]
        if busy:
            out["gpu_busy_percent"] = float(np.mean(busy))
        if vram:
            out["gpu_vram_mb"] = float(np.mean(vram))
        return out
