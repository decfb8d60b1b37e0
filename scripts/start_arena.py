#!/usr/bin/env python3
"""Start one topology as local processes (replaces the reference's docker compose files and
scripts/start-*.sh): each service is a child process; Ctrl-C stops them all.

  monolithic     replicas of :8100 (one per GPU, shared port)
  microservices  one classification gRPC service per GPU (:8201, :8211, ... on GPU 0, 1, ...) +
                 detection HTTP :8200 replicas (one per GPU) fanning crops over all classification services
                 (least-outstanding gRPC channel pool); --split puts detection on the first half of the
                 GPUs and classification on the second half
  triton         one model server per GPU (shared :8000/:8001/:8002, native KServe :8004 + 10 g) + one native
                 gateway per GPU on :8300 spreading requests over every model server (least outstanding)

Example: python scripts/start_arena.py --arch triton --gpus 1
"""
from __future__ import annotations

import argparse
import os
import signal
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


_next_cpu = [0]


def _envelope_cpus() -> list[int] | None:
    """``ARENA_SERVICE_CPUS=N``: every spawned service process (and its children: replicas, decode workers) is
    confined to N CPUs of its own, disjoint between services — the reference's per-container envelope of 2
    vCPU (experiment.yaml:250-267, docker-compose cpus: 2).  GPUs are not partitioned."""
    n = int(os.environ.get("ARENA_SERVICE_CPUS", "0") or 0)
    if n <= 0 or not hasattr(os, "sched_getaffinity"):
        return None
    allowed = sorted(os.sched_getaffinity(0))
    start = _next_cpu[0]
    if start + n > len(allowed):
        raise RuntimeError(f"ARENA_SERVICE_CPUS={n}: not enough CPUs for another service ({len(allowed)} allowed)")
    _next_cpu[0] = start + n
    return allowed[start:start + n]


def spawn(args, env, log_dir: Path, name: str):
    log = open(log_dir / f"{name}.log", "w")
    cpus = _envelope_cpus()
    if cpus is not None:
        print(f"[start_arena] {name}: CPUs {cpus}", flush=True)
    # affinity is set in the child before exec (the parent never initialises the GPU)
    pre = (lambda: os.sched_setaffinity(0, cpus)) if cpus is not None else None
    return subprocess.Popen([sys.executable, "-m", *args], env=env, stdout=log, stderr=subprocess.STDOUT, cwd=ROOT,
                            preexec_fn=pre)


def wait_http(url: str, timeout: float, procs) -> bool:
    import urllib.request

    t0 = time.time()
    while time.time() - t0 < timeout:
        if any(p.poll() is not None for p in procs):
            return False
        try:
            with urllib.request.urlopen(url, timeout=2) as r:
                if r.status == 200:
                    return True
        except OSError:
            pass
        time.sleep(0.5)
    return False


def wait_replicas(url: str, n: int, timeout: float, procs) -> bool:
    """Replicas sharing one port (SO_REUSEPORT): poll ``url`` on fresh connections until ``n`` distinct
    ``x-arena-replica`` tags have answered 200 (the port opens with the first replica; the others may still be
    starting)."""
    import urllib.request

    seen: set[str] = set()
    t0 = time.time()
    while time.time() - t0 < timeout:
        if any(p.poll() is not None for p in procs):
            return False
        try:
            with urllib.request.urlopen(url, timeout=2) as r:
                if r.status == 200:
                    seen.add(r.headers.get("x-arena-replica", ""))
        except OSError:
            pass
        if len(seen) >= n:
            return True
        time.sleep(0.05)
    return False


def classification_ports(n: int, base: int = 8201) -> list[int]:
    return [base + 10 * i for i in range(max(1, n))]


def plan_microservices(gpus: int, split: bool = False, cls_procs_per_gpu: int = 1) -> dict:
    """GPU assignment of the microservices arm: detection GPUs, classification (GPU, port) pairs —
    ``cls_procs_per_gpu`` classification processes per GPU (ports 8201+10*i+k), all behind the detection
    services' least-outstanding channel pool, so the per-crop Python gRPC work scales past one process."""
    if split and gpus >= 2:
        det = list(range(gpus // 2))
        cls = list(range(gpus // 2, gpus))
    else:
        det = list(range(max(1, gpus)))
        cls = list(range(max(1, gpus)))
    k = max(1, int(cls_procs_per_gpu))
    pairs = [(g, p + j) for g, p in zip(cls, classification_ports(len(cls))) for j in range(k)]
    return {"detection_gpus": det, "classification": pairs,
            "endpoint": ",".join(f"127.0.0.1:{p}" for _, p in pairs)}


def plan_triton(gpus: int, procs_per_gpu: int = 1, base_port: int | None = None) -> dict:
    """Process layout of the Triton arm on ``gpus`` GPUs: (gpu, k, native KServe port) per model-server process —
    ``procs_per_gpu`` per GPU on ports base + 10 g + k — and the gateway's upstream list over all of them."""
    base = int(base_port if base_port is not None else os.environ.get("ARENA_KSERVE_NATIVE_PORT", "8004"))
    ms = [(g, k, base + 10 * g + k) for g in range(max(1, gpus)) for k in range(max(1, procs_per_gpu))]
    return {"model_servers": ms, "upstreams": ",".join(f"127.0.0.1:{p}" for _, _, p in ms)}


def hw_queues_per_process(procs_on_gpu: int) -> int | None:
    """GPU_MAX_HW_QUEUES for each of ``procs_on_gpu`` GPU processes sharing one device (None: HIP's default 4).
    Five service processes x 4 hardware queues oversubscribed the device's queue slots: the firmware
    time-sliced them, GPU busy read 100 % at one user and P99 was 29 ms; capped at 2 queues per process,
    25 % busy and P99 6.3 ms, +48 % req/s at 10 users (profiles/serving_r2d/hwq/)."""
    n = int(procs_on_gpu)
    return None if n <= 3 else max(1, 10 // n)


def _queue_env(env: dict, procs_on_gpu: int) -> dict:
    """The children's environment with the queue cap applied.  ``ARENA_HW_QUEUES`` overrides the cap; an
    inherited ``GPU_MAX_HW_QUEUES`` does not (the GPU pool exports HIP's default 4 to every job)."""
    if env.get("ARENA_HW_QUEUES"):
        return dict(env, GPU_MAX_HW_QUEUES=str(int(env["ARENA_HW_QUEUES"])))
    q = hw_queues_per_process(procs_on_gpu)
    return env if q is None else dict(env, GPU_MAX_HW_QUEUES=str(q))


def start(arch: str, gpus: int, log_dir: Path, device: str = "gpu", repo: str = "model_repository",
          extra_env: dict | None = None, procs_per_gpu: int = 1, split: bool = False):
    env = dict(os.environ, PYTHONPATH=str(ROOT), HSA_ENABLE_IPC_MODE_LEGACY="0", ARENA_DEVICE=device,
               **(extra_env or {}))
    log_dir.mkdir(parents=True, exist_ok=True)
    _next_cpu[0] = 0  # CPU envelopes are allocated per arm
    procs = []
    if arch == "monolithic":
        procs.append(spawn(["inference_arena_amd.parallel.replicas", "--arch", "monolithic", "--gpus", str(gpus),
                            "--port", "8100", "--procs-per-gpu", str(procs_per_gpu)],
                           _queue_env(env, procs_per_gpu), log_dir, "monolithic"))
        ok = wait_replicas("http://127.0.0.1:8100/health", max(1, gpus) * max(1, procs_per_gpu), 600, procs)
    elif arch == "microservices":
        cls_k = int(os.environ.get("ARENA_CLS_PROCS_PER_GPU", "1"))
        plan = plan_microservices(gpus, split, cls_k)
        # GPU processes per device: detection + classification processes, unless they sit on disjoint GPUs
        env = _queue_env(env, max(procs_per_gpu, cls_k) if split and gpus >= 2 else procs_per_gpu + cls_k)
        for g, port in plan["classification"]:
            procs.append(spawn(["inference_arena_amd.server.classification_service"],
                               dict(env, PORT=str(port), ARENA_GPU=str(g)), log_dir,
                               f"classification_gpu{g}_{port}"))
        time.sleep(1)
        det = plan["detection_gpus"]
        procs.append(spawn(["inference_arena_amd.parallel.replicas", "--arch", "detection", "--gpus", str(len(det)),
                            "--first-gpu", str(det[0]), "--port", "8200", "--procs-per-gpu", str(procs_per_gpu)],
                           dict(env, CLASSIFICATION_GRPC_ENDPOINT=plan["endpoint"]), log_dir, "detection"))
        ok = wait_http("http://127.0.0.1:8200/health", 600, procs)
    elif arch == "triton":
        if not (Path(repo) / "yolov5n" / "config.pbtxt").exists():
            subprocess.run([sys.executable, str(ROOT / "scripts" / "upload_models.py"), "--repository", repo],
                           check=True, env=env)
        plan = plan_triton(gpus, procs_per_gpu)
        # one model-server process per GPU: each owns its device, pins itself to that GPU's
        # CPU share with a host plan sized for it (parallel/affinity.py rank_host_setup) and serves its own native
        # KServe endpoint; gRPC :8001 / HTTP :8000 / metrics :8002 are shared (SO_REUSEPORT) for Triton clients.
        # Its batches overlap in free slots, as the monolithic server's do (several processes per GPU keep it off)
        ms_env = _queue_env(dict(env, ARENA_LOCAL_WORLD=str(max(1, gpus))), procs_per_gpu)
        ms_env.setdefault("ARENA_BATCH_OVERLAP", "1" if procs_per_gpu <= 1 else "0")
        for g, k, port in plan["model_servers"]:
            procs.append(spawn(["inference_arena_amd.server.model_server", "--model-repository", repo, "--device",
                                device, "--gpu", str(g), "--native-http-port", str(port)],
                               dict(ms_env, ARENA_GPUS=str(g), ARENA_GPU=str(g)), log_dir, f"model_server_gpu{g}_{k}"))
        ok = all(wait_http(f"http://127.0.0.1:{port}/v2/health/ready", 600, procs)
                 for _, _, port in plan["model_servers"])
        if ok:
            # ARENA_GATEWAY_NATIVE (default 1): native gateway processes, one per GPU on :8300 (SO_REUSEPORT), each
            # spreading requests over every model server's native endpoint (least outstanding); 0 keeps the Python
            # gateway on gRPC :8001
            gw_native = os.environ.get("ARENA_GATEWAY_NATIVE", "1") != "0"
            # Python gateway processes (SO_REUSEPORT on :8300): ARENA_GATEWAY_PROCS, default procs_per_gpu (the
            # reference-shaped tensor mode is one GIL-bound process per gateway, ~15 ms CPU per request)
            gw_py = int(os.environ.get("ARENA_GATEWAY_PROCS", str(procs_per_gpu)))
            procs.append(spawn(["inference_arena_amd.parallel.replicas", "--arch", "gateway", "--gpus",
                                str(max(1, gpus) if gw_native else 1), "--port", "8300",
                                "--procs-per-gpu", str(1 if gw_native else gw_py)],
                               dict(env, TRITON_GRPC_ENDPOINT="127.0.0.1:8001", ARENA_DEVICE="cpu",
                                    TRITON_HTTP_ENDPOINT=plan["upstreams"],
                                    ARENA_GATEWAY_NATIVE="1" if gw_native else "0"), log_dir,
                               "gateway"))
            ok = wait_replicas("http://127.0.0.1:8300/health", max(1, gpus) if gw_native else gw_py, 300, procs)
    else:
        raise ValueError(arch)
    return procs, ok


def stop(procs) -> None:
    for p in reversed(procs):
        if p.poll() is None:
            p.send_signal(signal.SIGINT)
    for p in reversed(procs):
        try:
            p.wait(20)
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait(5)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--arch", required=True, choices=["monolithic", "microservices", "triton"])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--device", default="gpu", choices=["gpu", "cpu", "fake"],
                    help="fake: host-only stand-in engines (CPU tests of the process layout)")
    ap.add_argument("--logs", default="logs")
    ap.add_argument("--procs-per-gpu", type=int, default=1)
    ap.add_argument("--split", action="store_true",
                    help="microservices: detection and classification on disjoint GPU halves")
    a = ap.parse_args(argv)
    procs, ok = start(a.arch, a.gpus, Path(a.logs), a.device, procs_per_gpu=a.procs_per_gpu, split=a.split)
    print(f"{a.arch}: {'ready' if ok else 'FAILED (see ' + a.logs + ')'}", flush=True)
    try:
        while ok and all(p.poll() is None for p in procs):
            time.sleep(1)
    except KeyboardInterrupt:
        pass
    finally:
        stop(procs)
    return 0 if ok else 1


if __name__ == "__main__":
    raise SystemExit(main())
