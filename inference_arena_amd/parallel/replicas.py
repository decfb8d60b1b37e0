"""Launch N serving replicas (one process per GPU) on one node.

``launch(arch, n)`` starts ``server.replica`` N times with torchrun-style
environment (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR=127.0.0.1 /
MASTER_PORT) and ``HSA_ENABLE_IPC_MODE_LEGACY=0`` (dmabuf IPC, required by
RCCL on these hosts); replicas share the HTTP port via SO_REUSEPORT unless a
port stride is given.  ``wait_ready`` polls ``/health`` until every replica
answers; ``stop`` terminates the exact PIDs it started.

CLI: ``python -m inference_arena_amd.parallel.replicas --arch monolithic --gpus 8``.
"""
from __future__ import annotations

import argparse
import os
import signal
import socket
import subprocess
import sys
import time
from dataclasses import dataclass


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@dataclass
class Replicas:
    procs: list
    port: int
    stride: int

    def ports(self) -> list[int]:
        return [self.port + self.stride * r for r in range(len(self.procs))] if self.stride else [self.port]

    def alive(self) -> bool:
        return all(p.poll() is None for p in self.procs)

    def wait_ready(self, timeout: float = 300.0) -> bool:
        import urllib.request

        t0 = time.time()
        pending = set(self.ports())
        while pending and time.time() - t0 < timeout:
            if not self.alive():
                return False
            for p in list(pending):
                try:
                    with urllib.request.urlopen(f"http://127.0.0.1:{p}/health", timeout=2) as r:
                        if r.status == 200:
                            pending.discard(p)
                except OSError:
                    pass
            time.sleep(0.5)
        return not pending

    def stop(self, timeout: float = 20.0) -> None:
        for p in self.procs:
            if p.poll() is None:
                p.send_signal(signal.SIGINT)
        t0 = time.time()
        for p in self.procs:
            try:
                p.wait(max(0.1, timeout - (time.time() - t0)))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait(5)


def launch(arch: str, n: int, *, port: int = 8100, stride: int = 0, host: str = "127.0.0.1",
           env: dict | None = None, log_dir: str | None = None, procs_per_gpu: int = 1) -> Replicas:
    """``n`` GPUs x ``procs_per_gpu`` serving processes.  Several processes per GPU
    scale the CPU side (HTTP parsing, JPEG decode) while sharing the device; the
    start-up weight broadcast then runs over gloo, because one RCCL
    communicator cannot hold two ranks of the same GPU."""
    master = free_port()
    procs = []
    world = n * procs_per_gpu
    for r in range(world):
        e = dict(os.environ)
        e.update(env or {})
        e.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(world), "MASTER_ADDR": "127.0.0.1",
                  "MASTER_PORT": str(master), "HSA_ENABLE_IPC_MODE_LEGACY": "0",
                  "ARENA_PROCS_PER_GPU": str(procs_per_gpu)})
        out = open(os.path.join(log_dir, f"replica_{r}.log"), "w") if log_dir else subprocess.DEVNULL
        procs.append(subprocess.Popen([sys.executable, "-m", "inference_arena_amd.server.replica", "--arch", arch,
                                       "--host", host, "--port", str(port), "--port-stride", str(stride)],
                                      env=e, stdout=out, stderr=subprocess.STDOUT))
    return Replicas(procs, port, stride)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="monolithic")
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--port", type=int, default=8100)
    ap.add_argument("--stride", type=int, default=0)
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--procs-per-gpu", type=int, default=int(os.environ.get("ARENA_PROCS_PER_GPU", "1")))
    a = ap.parse_args(argv)
    rep = launch(a.arch, a.gpus, port=a.port, stride=a.stride, host=a.host, procs_per_gpu=a.procs_per_gpu)
    try:
        ok = rep.wait_ready()
        print(f"{a.gpus} GPU(s) x {a.procs_per_gpu} process(es) {'ready' if ok else 'FAILED'} on port(s) "
              f"{rep.ports()}", flush=True)
        while rep.alive():
            time.sleep(1)
    except KeyboardInterrupt:
        pass
    finally:
        rep.stop()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
