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
from dataclasses import dataclass, field


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@dataclass
class Replicas:
    procs: list
    port: int
    stride: int
    specs: list = None  # (argv, env, gpu, log path) per replica, for restarts
    restarts: int = 0
    stopping: bool = False
    # restart policy: the first restart of a replica is immediate, each further one waits backoff_s * 2^k
    # (capped at backoff_max_s); a replica that failed max_restarts times in a row (each run shorter than
    # healthy_s) is left down instead of crash-looping (every attempt initialises a GPU)
    max_restarts: int = 5
    backoff_s: float = 0.5
    backoff_max_s: float = 30.0
    healthy_s: float = 60.0
    given_up: set = field(default_factory=set)
    _fails: dict = field(default_factory=dict)
    _next: dict = field(default_factory=dict)
    _started: dict = field(default_factory=dict)

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

    def supervise(self) -> int:
        """Restart replicas that exited with a non-zero code (device fault: code 3) as fresh child
        processes on the same GPU, port and replica rank; returns the number restarted by this call."""
        n = 0
        if self.stopping or not self.specs:
            return 0
        now = time.time()
        for i, p in enumerate(self.procs):
            rc = p.poll()
            if rc is None or rc == 0 or i in self.given_up or now < self._next.get(i, 0.0):
                continue
            if now - self._started.get(i, 0.0) >= self.healthy_s:
                self._fails[i] = 0  # it served for a while before failing: not a crash loop
            k = self._fails.get(i, 0)
            if k >= self.max_restarts:
                self.given_up.add(i)
                print(f"replica {i}: exited rc={rc} after {k} restarts in a row; leaving it down", flush=True)
                continue
            argv, env, gpu, log = self.specs[i]
            e = dict(env)
            # the start-up process group is gone: the new process serves alone with the seeded weights, on
            # its original port and replica tag (ARENA_REPLICA_RANK; RANK is 0 in its one-process world)
            e.update({"RANK": "0", "LOCAL_RANK": "0", "WORLD_SIZE": "1", "ARENA_REPLICA_GPU": str(gpu),
                      "ARENA_REPLICA_RANK": env.get("ARENA_REPLICA_RANK", env.get("RANK", str(i))),
                      "ARENA_RESTARTED": str(self.restarts + 1)})
            e.pop("MASTER_PORT", None)
            out = open(log, "a") if log else None  # None: the supervisor's own stdout (its log file)
            self.procs[i] = subprocess.Popen(argv, env=e, stdout=out, stderr=subprocess.STDOUT)
            self._fails[i] = k + 1
            self._started[i] = now
            self._next[i] = now + min(self.backoff_max_s, self.backoff_s * 2 ** k)
            self.restarts += 1
            n += 1
        return n

    def stop(self, timeout: float = 20.0) -> None:
        self.stopping = True
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
           env: dict | None = None, log_dir: str | None = None, procs_per_gpu: int = 1,
           first_gpu: int = 0) -> Replicas:
    """``n`` GPUs x ``procs_per_gpu`` serving processes.  Several processes per GPU
    scale the CPU side (HTTP parsing, JPEG decode) while sharing the device; the
    start-up weight broadcast then runs over gloo, because one RCCL
    communicator cannot hold two ranks of the same GPU."""
    master = free_port()
    procs, specs = [], []
    world = n * procs_per_gpu
    for r in range(world):
        e = dict(os.environ)
        e.update(env or {})
        e.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(world), "MASTER_ADDR": "127.0.0.1",
                  "MASTER_PORT": str(master), "HSA_ENABLE_IPC_MODE_LEGACY": "0",
                  "ARENA_PROCS_PER_GPU": str(procs_per_gpu), "ARENA_FIRST_GPU": str(first_gpu),
                  # GPUs served on this node: each replica sizes its host threads for its share of the CPUs
                  # (parallel/affinity.py rank_host_setup)
                  "ARENA_LOCAL_WORLD": str(n)})
        log = os.path.join(log_dir, f"replica_{r}.log") if log_dir else None
        out = open(log, "w") if log else None  # None: the supervisor's own stdout (a failed start stays visible)
        argv = [sys.executable, "-m", "inference_arena_amd.server.replica", "--arch", arch, "--host", host,
                "--port", str(port), "--port-stride", str(stride)]
        procs.append(subprocess.Popen(argv, env=e, stdout=out, stderr=subprocess.STDOUT))
        specs.append((argv, e, first_gpu + r // procs_per_gpu, log))
    rep = Replicas(procs, port, stride, specs)
    rep._started = {i: time.time() for i in range(world)}
    return rep


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="monolithic")
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--port", type=int, default=8100)
    ap.add_argument("--stride", type=int, default=0)
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--procs-per-gpu", type=int, default=int(os.environ.get("ARENA_PROCS_PER_GPU", "1")))
    ap.add_argument("--first-gpu", type=int, default=int(os.environ.get("ARENA_FIRST_GPU", "0")))
    a = ap.parse_args(argv)
    rep = launch(a.arch, a.gpus, port=a.port, stride=a.stride, host=a.host, procs_per_gpu=a.procs_per_gpu,
                 first_gpu=a.first_gpu)
    try:
        ok = rep.wait_ready()
        print(f"{a.gpus} GPU(s) x {a.procs_per_gpu} process(es) {'ready' if ok else 'FAILED'} on port(s) "
              f"{rep.ports()}", flush=True)
        while True:
            if rep.supervise():
                print(f"restarted replica(s); {rep.restarts} restart(s) so far", flush=True)
            if all(p.poll() == 0 for p in rep.procs):
                break
            time.sleep(0.5)
    except KeyboardInterrupt:
        pass
    finally:
        rep.stop()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
