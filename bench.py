#!/usr/bin/env python3
"""Headline benchmark: whole-node req/s + per-request P50/P99 end-to-end latency of the
YOLOv5n -> MobileNetV2 request pipeline on 1..8 MI355X (BASELINE.json metric).

Metric definition (reference protocol: closed-loop users sending JPEG uploads and timing
each request end to end, reference experiment.yaml:178-181,300-318):

* every rank (one per GPU) runs ``--users`` (256) closed-loop clients.  A client sends one
  encoded JPEG of the curated synthetic workload (3-5 detections per image, mean 4: the
  reference's thesis test-set protocol), waits for its result and immediately sends the
  next one.  A request is timed from the moment its JPEG bytes are handed to the server
  side to the moment its detections + classifications are back on the host:
    JPEG decode (multi-process decode pool, spawned workers) -> native dynamic batcher
    (csrc/runtime/batcher.cpp, max_batch 32) -> H2D -> letterbox -> YOLOv5nu -> decode ->
    NMS -> crop gather -> MobileNetV2 -> top-5 -> D2H -> per-request result split.
* precision: ``--dtype fp32`` (default) runs the exact-fp32 kernels, the reference's fp32
  ONNX Runtime numerics (reference experiment.yaml:202,207,220,225); ``bf16`` the tuned
  bf16 kernels.
* steady state: the clients run continuously from the warm-up into the timed window, so
  the window contains no pipeline fill or drain.  A "step" is ``--step-batches`` (8) dynamic
  batches of ``--batch`` (32) = 256 completed requests (a 32-request step made a 20-step
  window ~85 ms long, where one host hiccup moved the result by 20 %): ``--warmup`` steps
  complete untimed, then a barrier + device sync open the window, the window closes (device
  sync + barrier) once exactly ``--steps`` more steps have completed on the rank.
  ``value`` = steps * requests per step * world / max-over-ranks window.
  P50/P99 are per-request end-to-end latencies of the requests completed in the window.

Multi-GPU: ``--gpus N`` under torchrun (RANK/LOCAL_RANK/WORLD_SIZE from the environment)
runs one rank per GPU over RCCL (rank 0's folded weights are broadcast over xGMI); run
without WORLD_SIZE and N > 1 it launches ``torch.distributed.run`` itself as a child
process (before any GPU call) and exits with its code.

Secondary keys: ``engine_req_s`` (device pipeline fed pre-decoded images, same dtype),
``bf16`` (the same end-to-end measurement on the bf16 kernels; on by default,
``--no-secondary-bf16`` skips it), bs=1 latency (one client).
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import subprocess
import sys
import threading
import time
from pathlib import Path

os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC for RCCL on these hosts

import numpy as np  # noqa: E402

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = "req/sec (whole node) + P50/P99 e2e latency, YOLOv5n→MobileNetV2 at 1/2/4/8 GPU"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def host_cpus() -> int:
    """CPUs this job may use: the affinity mask, capped by a cgroup-v2 CPU quota (cpu.max) when one is set —
    on the GPU pool the mask shows the whole machine while the quota is the job's share."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 8)
    try:
        quota, period = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) / int(period))))
    except (OSError, ValueError):
        pass
    return n


def self_launch(argv: list[str], n: int) -> int:
    """Re-run this script under torch.distributed.run with N ranks (child process, no exec)."""
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), str(Path(__file__).resolve()), *argv]
    log("launching", " ".join(cmd))
    return subprocess.call(cmd, env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0"))


def load_workload(pipe, info, n_images: int, seed: int, dtype: str):
    """The curated workload for this precision (curated with the same pipeline: 3-5 detections per image)."""
    from inference_arena_amd.data.curator import CurationConfig, DatasetManifest, curate, load_manifest_images
    from inference_arena_amd.parallel.dist import broadcast_object

    sfx = "" if dtype == "fp32" else f"_{dtype}"
    path = ROOT / "data" / "synthetic_set" / f"manifest_w{seed}_n{n_images}{sfx}.json"
    man = None
    if info.is_main:
        if path.exists():
            man = DatasetManifest.load(path)
        else:
            t = time.time()

            def counter(imgs):
                return [len(r) for r in pipe.infer(imgs)]

            _, man = curate(counter, CurationConfig(target_count=n_images), log=log)
            man.config["weight_seed"] = seed
            try:
                man.save(path)
            except OSError:
                pass
            log(f"curated {len(man.images)} images in {time.time() - t:.1f}s: {man.statistics}")
    man = broadcast_object(man.to_dict() if man is not None else None, info)
    man = DatasetManifest(**man)
    return load_manifest_images(man), man


class ClosedLoop:
    """``users`` closed-loop clients: JPEG -> decode pool -> native batcher -> result -> next request."""

    def __init__(self, pool, batcher, jpegs: list[bytes], users: int, offset: int = 0):
        self.pool, self.batcher, self.jpegs, self.users = pool, batcher, jpegs, users
        self.lock = threading.Lock()
        self.cv = threading.Condition(self.lock)
        self.done = 0
        self.errors = 0
        self.lat: list[float] = []    # per completed request, completion order
        self.crops: list[int] = []
        self.batch: list[int] = []
        self.next_img = offset
        self.running = False
        self.in_flight = 0

    def _issue(self) -> None:
        with self.lock:
            if not self.running:
                return
            i = self.next_img % len(self.jpegs)
            self.next_img += 1
            self.in_flight += 1
        self.pool.submit(self.jpegs[i], time.perf_counter(), self._decoded)

    def _decoded(self, t0, img, err) -> None:
        if err is not None or img is None:
            self._complete(t0, None)
            return

        def done(d, t0=t0):
            self._complete(t0, d)

        if self.batcher.enqueue(img, done) < 0:
            self._complete(t0, None)

    def _complete(self, t0, d) -> None:
        t1 = time.perf_counter()
        with self.lock:
            self.in_flight -= 1
            if d is None or d.get("error"):
                self.errors += 1
            else:
                self.lat.append(t1 - t0)
                self.crops.append(int(d["topk_idx"].shape[0]))
                self.batch.append(int(d["batch_size"]))
                self.done += 1
            self.cv.notify_all()
        self._issue()

    def start(self) -> None:
        self.running = True
        for _ in range(self.users):
            self._issue()

    def wait_for(self, n: int, timeout: float = 600.0) -> None:
        deadline = time.time() + timeout
        with self.lock:
            while self.done < n:
                if self.errors > 100 and self.done == 0:
                    raise RuntimeError(f"{self.errors} failed requests and none completed")
                left = deadline - time.time()
                if left <= 0:
                    raise TimeoutError(f"only {self.done}/{n} requests completed")
                self.cv.wait(min(left, 1.0))

    def stop(self) -> None:
        with self.lock:
            self.running = False
        deadline = time.time() + 60
        with self.lock:
            while self.in_flight > 0 and time.time() < deadline:
                self.cv.wait(0.5)


def engine_throughput(pipe, images, B: int, batches: int) -> float:
    """Device pipeline alone (pre-decoded images, pipelined submit/collect): requests/s between the
    completion of the first ``depth`` batches and the last one (fill and drain excluded)."""
    depth = pipe.ex.num_slots()
    n = len(images)
    q, done_t = [], []
    k = 0
    for st in range(batches + depth):
        q.append(pipe.ex.submit([images[(k + i) % n] for i in range(B)]))
        k += B
        if len(q) == depth:
            pipe.ex.collect(q.pop(0))
            done_t.append(time.perf_counter())
    while q:
        pipe.ex.collect(q.pop(0))
        done_t.append(time.perf_counter())
    return (len(done_t) - depth) * B / (done_t[-1] - done_t[depth - 1])


def measure(pipe, pool, jpegs, a, info, D, torch):
    """The closed-loop end-to-end window on one rank; returns (window seconds, latencies, crops, batches)."""
    from inference_arena_amd.ops import native

    C = native()
    B = a.batch
    R = B * a.step_batches  # requests per step
    batcher = C.DynamicBatcher([pipe.ex], {"max_batch": B, "max_queue_delay_us": a.queue_delay_us,
                                           "max_queue_size": 0})
    loop = ClosedLoop(pool, batcher, jpegs, a.users, offset=(info.rank * 37) % len(jpegs))
    gc.collect()
    gc.freeze()  # the long-lived heap (models, workload) leaves the collector's generations before the loop runs
    loop.start()
    try:
        # W warm-up steps at least; the closed loop also has to leave its start-up transient (all users
        # arrive at once, first graph replays) before the window opens: >= 4 requests per user and
        # --min-warmup-s seconds, so the window's value does not depend on --steps / --warmup
        tw = time.perf_counter()
        loop.wait_for(max(a.warmup * R, 4 * a.users))
        while time.perf_counter() - tw < a.min_warmup_s:
            time.sleep(0.05)
        D.barrier(info)
        torch.cuda.synchronize()
        gc.disable()  # no collector pauses inside the window (the loop allocates per request)
        with loop.lock:
            c0 = loop.done
        t0 = time.perf_counter()
        loop.wait_for(c0 + a.steps * R)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        gc.enable()
        D.barrier(info)
    finally:
        gc.enable()
        loop.stop()
        batcher.shutdown()
    lat = loop.lat[c0:c0 + a.steps * R]
    crops = loop.crops[c0:c0 + a.steps * R]
    bs = loop.batch[c0:c0 + a.steps * R]
    return t1 - t0, lat, crops, bs, loop.errors


def bs1_latency(pipe, pool, jpegs, n: int, a):
    """One client, sequential requests: the single-request (monolithic 1-user) latency floor, end to end."""
    from inference_arena_amd.ops import native

    batcher = native().DynamicBatcher([pipe.ex], {"max_batch": 1, "max_queue_delay_us": 0})
    loop = ClosedLoop(pool, batcher, jpegs, 1)
    loop.start()
    try:
        loop.wait_for(5 + n)
    finally:
        loop.stop()
        batcher.shutdown()
    return loop.lat[5:5 + n]


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30,
                    help="timed steps (a step = --step-batches x --batch completed requests)")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--min-warmup-s", type=float, default=2.0, help="minimum warm-up time of the closed loop")
    ap.add_argument("--batch", type=int, default=32, help="dynamic batcher max_batch")
    ap.add_argument("--step-batches", type=int, default=8, help="batches of --batch requests per step")
    # 256: enough requests in flight that every dynamic batch is full (4 staging slots x 32 on the device plus
    # the decode pipeline); 192 left the batcher short (mean batch 30.5: 7.0k vs 7.5k req/s, P50 25 vs 33 ms;
    # profiles/r2_final_bench_20steps.json vs r2_bench_users256.json)
    ap.add_argument("--users", type=int, default=256, help="closed-loop clients per GPU")
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--decode-workers", type=int, default=0, help="JPEG decode processes per rank (0: auto)")
    ap.add_argument("--queue-delay-us", type=int, default=2000)
    ap.add_argument("--jpeg-quality", type=int, default=90)
    ap.add_argument("--seed", type=int, default=0, help="weight seed")
    ap.add_argument("--images", type=int, default=100, help="curated workload size")
    ap.add_argument("--bs1-requests", type=int, default=50)
    ap.add_argument("--engine-batches", type=int, default=40, help="batches for the engine-only secondary key")
    ap.add_argument("--secondary-bf16", action=argparse.BooleanOptionalAction, default=True,
                    help="also measure the bf16 kernels (secondary key 'bf16': e2e, P50/P99, engine req/s)")
    ap.add_argument("--crop-cap", type=int, default=None)
    a = ap.parse_args(argv)
    raw_argv = list(sys.argv[1:] if argv is None else argv)

    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return self_launch(raw_argv, a.gpus)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != a.gpus:
        log(f"error: --gpus {a.gpus} but WORLD_SIZE={world}")
        return 2

    # decode workers are spawned before this process touches the GPU
    from inference_arena_amd.server.decode_pool import ProcessDecodePool

    ncpu = host_cpus()
    # 10 decode processes (~8.5k decodes/s) keep a GPU's engine (~7k req/s fp32) fed; more of them compete with
    # the batcher / packing threads for the box's CPU share and lowered the e2e rate (16-CPU box: 15 workers
    # 6.0-6.4k req/s, 8-10 workers 6.78k; profiles/r2_decode_workers_sweep.md)
    workers = a.decode_workers or max(2, min(10, ncpu // max(1, world) - 1))
    pool = ProcessDecodePool(workers=workers, slots=max(256, a.users + 64))

    import torch

    from inference_arena_amd.data.synthetic import encode_jpeg
    from inference_arena_amd.engine.pipeline import GpuPipeline
    from inference_arena_amd.models.zoo import default_models
    from inference_arena_amd.parallel import dist as D

    info = D.init_from_env(os.environ.get("ARENA_DIST_BACKEND") or None)
    assert info.world == a.gpus, (info.world, a.gpus)
    # ARENA_SHARED_GPU=1 (+ ARENA_DIST_BACKEND=gloo): rehearse the N-rank path on a 1-GPU box, every rank on
    # device 0 (the driver's 8-GPU run uses one GPU per rank over RCCL)
    dev = 0 if os.environ.get("ARENA_SHARED_GPU") == "1" else info.local_rank
    torch.cuda.set_device(dev)
    torch.set_num_threads(2)
    try:
        t0 = time.time()
        yolo, mnet = default_models(a.seed)
        buckets = sorted({1, a.batch})
        pipe = GpuPipeline(yolo, mnet, device=dev, buckets=buckets, crop_cap_per_image=a.crop_cap,
                           dtype=a.dtype)
        if info.world > 1:
            # rank 0's folded weights, broadcast with RCCL over xGMI straight into each replica's GPU memory
            blob = D.broadcast_blob_device(pipe.program.weights if info.is_main else None, info)
            if blob.is_cuda:
                pipe.ex.set_weights_device(blob.data_ptr(), blob.numel())
            else:
                pipe.ex.set_weights(blob.cpu().numpy())
            torch.cuda.synchronize()
        log(f"[rank {info.rank}/{info.world} {info.backend}] {a.dtype} pipeline ready in {time.time() - t0:.1f}s; "
            f"arena MB {({b: round(v / 2**20, 1) for b, v in pipe.arena_bytes.items()})}; decode workers {workers}")

        images, man = load_workload(pipe, info, a.images, a.seed, a.dtype)
        # the uploads are the JPEGs the workload was curated on (manifest config.jpeg_quality)
        a.jpeg_quality = int(man.config.get("jpeg_quality", a.jpeg_quality))
        jpegs = [encode_jpeg(im, a.jpeg_quality) for im in images]

        window, lat, crops, bs, errs = measure(pipe, pool, jpegs, a, info, D, torch)
        t_max = D.allreduce_max(window, info)

        eng = engine_throughput(pipe, images, a.batch, a.engine_batches) if a.engine_batches > 0 else None
        bs1 = bs1_latency(pipe, pool, jpegs, a.bs1_requests, a) if (info.is_main and a.bs1_requests > 0) else []
        sec = {}
        if a.secondary_bf16 and a.dtype != "bf16":
            alt = GpuPipeline(yolo, mnet, device=dev, buckets=buckets, crop_cap_per_image=a.crop_cap,
                              dtype="bf16")
            w2, lat2, _, _, _ = measure(alt, pool, jpegs, a, info, D, torch)
            w2 = D.allreduce_max(w2, info)
            sec = {"bf16": {"value": round(a.steps * a.batch * a.step_batches * info.world / w2, 2),
                            "p50_ms": round(float(np.percentile(lat2, 50)) * 1e3, 3),
                            "p99_ms": round(float(np.percentile(lat2, 99)) * 1e3, 3),
                            "engine_req_s": round(engine_throughput(alt, images, a.batch, a.engine_batches), 1)}}

        all_lat = D.allgather_floats(lat, info)
        all_crops = D.allgather_floats([float(c) for c in crops], info)
        all_eng = D.allgather_floats([eng or 0.0], info)
        all_err = D.allgather_floats([float(errs)], info)
        D.barrier(info)
        if info.is_main:
            flat = np.asarray([x for lst in all_lat for x in lst]) * 1e3
            total_req = a.steps * a.batch * a.step_batches * info.world
            fan = float(np.sum([x for lst in all_crops for x in lst]) / max(1, len(flat)))
            out = {
                "metric": METRIC,
                "value": round(total_req / t_max, 2),
                "unit": "req/s",
                "n_gpus": info.world,
                "steps": a.steps,
                "warmup": a.warmup,
                "ms_per_step": round(t_max / a.steps * 1e3, 4),
                "higher_is_better": True,
                "scaling": "weak",
                "vs_baseline": None,
                "dtype": a.dtype,
                "data": ("synthetic COCO-shaped RGB images encoded as JPEG q%d (curated to 3-5 detections, mean "
                         "fan-out %.2f); random-init YOLOv5nu + MobileNetV2 weights; per-request end to end: JPEG "
                         "decode + dynamic batching + full device pipeline + result split, %d closed-loop users/GPU"
                         % (a.jpeg_quality, fan, a.users)),
                "config": {
                    "model": "YOLOv5nu(640)->MobileNetV2(224)",
                    "global_batch": a.batch * info.world,
                    "seq_len": None,
                    "parallelism": f"dp{info.world}",
                    "per_gpu_batch": a.batch,
                    "requests_per_step_per_gpu": a.batch * a.step_batches,
                    "users_per_gpu": a.users,
                    "image_size": 640,
                    "crop_size": 224,
                    "decode_workers_per_gpu": workers,
                    "workload": {"images": len(images), "distribution": man.distribution,
                                 "mean_detections": man.statistics.get("mean_detections")},
                },
                "p50_ms": round(float(np.percentile(flat, 50)), 3),
                "p99_ms": round(float(np.percentile(flat, 99)), 3),
                "latency": "per-request end to end (JPEG bytes in -> results out)",
                "mean_crops_per_request": round(fan, 3),
                "mean_batch": round(float(np.mean(bs)), 2) if bs else None,
                "errors": int(sum(x for lst in all_err for x in lst)),
                "engine_req_s": round(float(sum(x for lst in all_eng for x in lst)), 1) if eng else None,
                "bs1_p50_ms": round(float(np.percentile(bs1, 50)) * 1e3, 3) if bs1 else None,
                "bs1_p99_ms": round(float(np.percentile(bs1, 99)) * 1e3, 3) if bs1 else None,
                "world_size_checked": info.world,
            }
            out.update(sec)
            print(json.dumps(out), flush=True)
    finally:
        pool.close()
    D.shutdown(info)
    return 0


if __name__ == "__main__":
    sys.exit(main())
