#!/usr/bin/env python3
"""Headline benchmark: whole-node req/s + per-request P50/P99 end-to-end latency of the
YOLOv5n -> MobileNetV2 ``POST /predict`` pipeline on 1..8 MI355X (BASELINE.json metric).

Metric definition (reference protocol: closed-loop users sending JPEG uploads and timing each
request end to end, reference experiment.yaml:178-181,300-318; the /predict handler of
architectures/monolithic/app/main.py:102-159):

* every rank (one per GPU) serves the monolithic arm behind the native HTTP/1.1 front end
  (``--path http``, default: csrc/runtime/http_front.cpp on a loopback port) and drives it with
  ``--users`` (256) closed-loop clients of the native load generator (csrc/runtime/http_loadgen.cpp:
  keep-alive connections, multipart uploads of the curated workload, 3-5 detections per image).  A
  request is timed from the moment its upload starts on the client to the moment the client has
  parsed the complete JSON response:
    HTTP + multipart parse -> JPEG decode (spawned decode processes, shared memory) -> native dynamic
    batcher (max_batch 32) -> H2D -> letterbox -> YOLOv5nu -> decode -> NMS -> crop gather ->
    MobileNetV2 -> top-5 -> D2H -> JSON response (the reference's schema) -> client.
  ``--path inproc`` measures the same pipeline without the HTTP layer (JPEG bytes handed to the decode
  pool, results read from the batcher callback); it is also reported as the secondary key ``inproc``.
* precision: ``--dtype fp32`` (default) runs the fp32-accurate kernels, the reference's fp32 ONNX
  Runtime numerics (reference experiment.yaml:202,207,220,225); ``bf16`` the tuned bf16 kernels.
* steady state: the clients run continuously from the warm-up into the timed window, so the window
  contains no pipeline fill or drain.  A "step" is ``--step-batches`` (32) dynamic batches of
  ``--batch`` (32) = 1024 completed requests: ``--warmup`` steps complete untimed, then a barrier +
  device sync open the window, the window closes (device sync + barrier) once exactly ``--steps`` more
  steps have completed on the rank.  ``value`` = steps * requests per step * world / max-over-ranks
  window.  P50/P99 are per-request end-to-end latencies of the requests completed in the window.
* reference load levels: rank 0 also reports P50/P99 and req/s at 1, 10 and 100 closed-loop users
  (``--latency-levels``) next to the saturation point.

Multi-GPU: ``--gpus N`` under torchrun (RANK/LOCAL_RANK/WORLD_SIZE from the environment) runs one rank
per GPU over RCCL: rank 0's folded weights are broadcast over xGMI into every replica's GPU memory and
every rank's device weights are hashed and compared (``weights_verified``).  Each rank pins itself and
its decode processes to its GPU's NUMA-local CPU share (parallel/affinity.py).  Run without WORLD_SIZE
and N > 1, bench.py launches ``torch.distributed.run`` itself as a child process (before any GPU call)
and exits with its code.

Secondary keys: ``inproc`` (same pipeline, no HTTP layer), ``engine_req_s`` (device pipeline fed
pre-decoded images), ``bf16`` (the end-to-end measurement on the bf16 kernels, in process),
``levels`` (1/10/100 users), ``per_rank_req_s``, ``cpu_share`` per rank.

``--fake-engine`` replaces the GPU pipeline by the host-only EchoInstance (CPU tests of the whole
harness, including the N-rank path over gloo: ARENA_DIST_BACKEND=gloo).
"""
from __future__ import annotations

import argparse
import gc
import hashlib
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


def http_request(jpeg: bytes) -> bytes:
    """The upload a reference client sends: POST /predict, multipart/form-data field ``file``."""
    from inference_arena_amd.server.multipart import encode_multipart

    body, ctype = encode_multipart("file", jpeg, filename="image.jpg", content_type="image/jpeg")
    return (f"POST /predict HTTP/1.1\r\nHost: 127.0.0.1\r\nContent-Type: {ctype}\r\n"
            f"Content-Length: {len(body)}\r\n\r\n").encode() + body


class ClosedLoop:
    """``users`` in-process closed-loop clients: JPEG -> decode pool -> native batcher -> result -> next."""

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

    def completed(self) -> int:
        with self.lock:
            return self.done

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


def engine_throughput(ex, images, B: int, batches: int) -> float:
    """Device pipeline alone (pre-decoded images, pipelined submit/collect): requests/s between the
    completion of the first ``depth`` batches and the last one (fill and drain excluded)."""
    depth = ex.num_slots()
    n = len(images)
    q, done_t = [], []
    k = 0
    for st in range(batches + depth):
        q.append(ex.submit([images[(k + i) % n] for i in range(B)]))
        k += B
        if len(q) == depth:
            ex.collect(q.pop(0))
            done_t.append(time.perf_counter())
    while q:
        ex.collect(q.pop(0))
        done_t.append(time.perf_counter())
    return (len(done_t) - depth) * B / (done_t[-1] - done_t[depth - 1])


def _window(a, info, D, sync, completed, wait_until, users: int):
    """Warm-up (>= --warmup steps, >= 4 requests per user, >= --min-warmup-s), barrier + sync, then the window
    of exactly --steps steps; returns (seconds, first completion index of the window)."""
    R = a.batch * a.step_batches
    tw = time.perf_counter()
    wait_until(max(a.warmup * R, 4 * users))
    while time.perf_counter() - tw < a.min_warmup_s:
        time.sleep(0.05)
    D.barrier(info)
    sync()
    gc.disable()  # no collector pauses inside the window
    try:
        c0 = completed()
        t0 = time.perf_counter()
        wait_until(c0 + a.steps * R)
        sync()
        t1 = time.perf_counter()
    finally:
        gc.enable()
    D.barrier(info)
    return t1 - t0, c0


def batcher_config(a) -> dict:
    # idle delay 100 us: a lone request is not held for the full queue delay (the 1/10-user levels); under
    # load the device is always busy and batches grow over the 2 ms busy delay (batcher.h)
    return {"max_batch": a.batch, "max_queue_delay_us": a.queue_delay_us, "idle_queue_delay_us": 100,
            "max_queue_size": 0}


def measure_http(port: int, reqs: list[bytes], a, info, D, sync, users: int):
    """Closed-loop HTTP window on one rank: (seconds, latencies s, detections, statuses)."""
    from inference_arena_amd.ops import native

    lg = native().HttpLoadGen({"host": "127.0.0.1", "port": port, "users": users,
                               "threads": max(1, min(a.lg_threads, users))}, reqs)
    lg.start()

    def wait_until(n):
        if not lg.wait_completed(n, 600.0):
            raise TimeoutError(f"HTTP load generator: {lg.completed()}/{n} responses "
                               f"({lg.connect_failures()} failed connects)")
    try:
        window, c0 = _window(a, info, D, sync, lg.completed, wait_until, users)
    finally:
        lg.stop(60.0)
    r = lg.records(c0, c0 + a.steps * a.batch * a.step_batches)
    return window, r["latency"].astype(np.float64), r["dets"].astype(np.int64), r["status"].astype(np.int64)


def measure_inproc(ex, pool, jpegs, a, info, D, sync):
    """The closed-loop window without the HTTP layer: (seconds, latencies, crops, batch sizes, errors)."""
    from inference_arena_amd.ops import native

    batcher = native().DynamicBatcher([ex], batcher_config(a))
    loop = ClosedLoop(pool, batcher, jpegs, a.users, offset=(info.rank * 37) % len(jpegs))
    gc.collect()
    gc.freeze()
    loop.start()
    try:
        window, c0 = _window(a, info, D, sync, loop.completed, loop.wait_for, a.users)
    finally:
        loop.stop()
        batcher.shutdown()
    n = a.steps * a.batch * a.step_batches
    return window, loop.lat[c0:c0 + n], loop.crops[c0:c0 + n], loop.batch[c0:c0 + n], loop.errors


def latency_levels(port: int, reqs: list[bytes], levels: list[int], a) -> dict:
    """P50/P99/req/s at the reference's closed-loop user levels (one rank's front end, short phases)."""
    from inference_arena_amd.ops import native

    out = {}
    for u in levels:
        n_warm, n_meas = max(30, 3 * u), max(300, 20 * u)
        lg = native().HttpLoadGen({"host": "127.0.0.1", "port": port, "users": u, "threads": max(1, min(2, u))},
                                  reqs)
        lg.start()
        try:
            if not lg.wait_completed(n_warm + n_meas, 300.0):
                raise TimeoutError(f"level {u}: {lg.completed()} responses")
        finally:
            lg.stop(60.0)
        r = lg.records(n_warm, n_warm + n_meas)
        lat = r["latency"].astype(np.float64) * 1e3
        t = r["t_done"]
        out[str(u)] = {"req_s": round(float((len(t) - 1) / max(1e-9, t[-1] - t[0])), 1),
                       "p50_ms": round(float(np.percentile(lat, 50)), 3),
                       "p99_ms": round(float(np.percentile(lat, 99)), 3),
                       "errors": int((r["status"] != 200).sum())}
    return out


class FakeEngine:
    """Host-only stand-in for the GPU pipeline (--fake-engine): the EchoInstance answers every image with a
    deterministic set of detections after ``latency_us``; the weight blob is a seeded random byte string."""

    def __init__(self, batch: int, seed: int):
        from inference_arena_amd.ops import native

        self.ex = native().EchoInstance(4, batch, 4, 1500)
        self.weights = np.random.default_rng(seed).integers(0, 256, 1 << 20, dtype=np.uint8)
        self.arena_bytes = {}

    def weights_host(self) -> bytes:
        return self.weights.tobytes()


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30,
                    help="timed steps (a step = --step-batches x --batch completed requests)")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--min-warmup-s", type=float, default=2.0, help="minimum warm-up time of the closed loop")
    ap.add_argument("--batch", type=int, default=32, help="dynamic batcher max_batch")
    ap.add_argument("--step-batches", type=int, default=32,
                    help="batches of --batch requests per step (32 x 32 = 1024 requests: ~0.1 s per step, so the "
                         "timed window is seconds rather than a fraction of one)")
    # 256: enough requests in flight that every dynamic batch is full (4 staging slots x 32 on the device plus
    # the decode pipeline); 192 left the batcher short (mean batch 30.5: 7.0k vs 7.5k req/s, P50 25 vs 33 ms;
    # profiles/r2_final_bench_20steps.json vs r2_bench_users256.json)
    ap.add_argument("--users", type=int, default=256, help="closed-loop clients per GPU")
    ap.add_argument("--path", default="http", choices=["http", "inproc"],
                    help="http: clients upload over HTTP to the native front end (headline); inproc: no HTTP layer")
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--decode-workers", type=int, default=0, help="JPEG decode processes per rank (0: auto)")
    ap.add_argument("--http-threads", type=int, default=4, help="epoll I/O threads of the native front end")
    ap.add_argument("--lg-threads", type=int, default=2, help="load-generator threads per rank")
    ap.add_argument("--queue-delay-us", type=int, default=2000)
    ap.add_argument("--jpeg-quality", type=int, default=90)
    ap.add_argument("--seed", type=int, default=0, help="weight seed")
    ap.add_argument("--images", type=int, default=100, help="curated workload size")
    ap.add_argument("--latency-levels", default="1,10,100", help="closed-loop user levels for P50/P99 ('' = skip)")
    ap.add_argument("--level-delay-us", type=int, default=500, help="batcher busy delay of the latency levels")
    ap.add_argument("--engine-batches", type=int, default=40, help="batches for the engine-only secondary key")
    ap.add_argument("--secondary-inproc", action=argparse.BooleanOptionalAction, default=True,
                    help="also measure the pipeline without the HTTP layer (secondary key 'inproc')")
    ap.add_argument("--secondary-bf16", action=argparse.BooleanOptionalAction, default=True,
                    help="also measure the bf16 kernels (secondary key 'bf16': e2e in process, engine req/s)")
    ap.add_argument("--crop-cap", type=int, default=None)
    ap.add_argument("--fake-engine", action="store_true", help="host-only EchoInstance instead of the GPU (CPU tests)")
    a = ap.parse_args(argv)
    raw_argv = list(sys.argv[1:] if argv is None else argv)

    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return self_launch(raw_argv, a.gpus)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != a.gpus:
        log(f"error: --gpus {a.gpus} but WORLD_SIZE={world}")
        return 2
    local_rank = int(os.environ.get("LOCAL_RANK", os.environ.get("RANK", "0")))
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))

    # this rank's host CPUs next to its GPU (sysfs only: nothing has touched the GPU yet); the decode workers
    # are spawned after the pin and inherit it
    from inference_arena_amd.parallel.affinity import pin, rank_cpu_share

    share = rank_cpu_share(local_rank, local_world) if not a.fake_engine else None
    pinned = pin(share)
    ncpu = host_cpus()
    from inference_arena_amd.server.decode_pool import ProcessDecodePool, prestart

    prestart()
    # 10 decode processes (~8.5k decodes/s) keep a GPU's engine fed; more of them compete with the batcher /
    # HTTP threads for the box's CPU share (16-CPU box: 15 workers 6.0-6.4k req/s, 8-10 workers 6.78k;
    # profiles/r2_decode_workers_sweep.md)
    workers = a.decode_workers or max(2, min(10, ncpu // max(1, world if not pinned else 1) - 1))
    pool = ProcessDecodePool(workers=workers, slots=max(256, a.users + 64), native=a.path == "http",
                             cpus=share if pinned else None)

    torch = None
    if not a.fake_engine:
        import torch

    from inference_arena_amd.data.synthetic import encode_jpeg, synthetic_images
    from inference_arena_amd.ops import native
    from inference_arena_amd.parallel import dist as D

    backend = os.environ.get("ARENA_DIST_BACKEND") or ("gloo" if a.fake_engine else None)
    info = D.init_from_env(backend)
    assert info.world == a.gpus, (info.world, a.gpus)
    # ARENA_SHARED_GPU=1 (+ ARENA_DIST_BACKEND=gloo): rehearse the N-rank path on a 1-GPU box, every rank on
    # device 0 (the driver's 8-GPU run uses one GPU per rank over RCCL)
    dev = 0 if os.environ.get("ARENA_SHARED_GPU") == "1" else info.local_rank

    def sync():
        if torch is not None:
            torch.cuda.synchronize()

    fe = None
    try:
        t0 = time.time()
        if a.fake_engine:
            pipe = FakeEngine(a.batch, a.seed)
            blob0 = pipe.weights
            if info.world > 1:
                pipe.weights = D.broadcast_blob(blob0 if info.is_main else None, info).copy()
                if os.environ.get("ARENA_TEST_CORRUPT_WEIGHTS") == str(info.rank):  # the check's own test
                    pipe.weights[123] ^= 1
            ex = pipe.ex
            digest = hashlib.sha256(pipe.weights_host()).hexdigest()
        else:
            from inference_arena_amd.engine.pipeline import GpuPipeline
            from inference_arena_amd.models.zoo import default_models

            torch.cuda.set_device(dev)
            torch.set_num_threads(2)
            yolo, mnet = default_models(a.seed)
            buckets = sorted({1, a.batch})
            pipe = GpuPipeline(yolo, mnet, device=dev, buckets=buckets, crop_cap_per_image=a.crop_cap, dtype=a.dtype)
            blob0 = pipe.program.weights
            if info.world > 1:
                # rank 0's folded weights, broadcast with RCCL over xGMI straight into each replica's GPU memory
                blob = D.broadcast_blob_device(blob0 if info.is_main else None, info)
                if blob.is_cuda:
                    pipe.ex.set_weights_device(blob.data_ptr(), blob.numel())
                else:
                    pipe.ex.set_weights(blob.cpu().numpy())
                torch.cuda.synchronize()
            ex = pipe.ex
            digest = hashlib.sha256(ex.weights_host()).hexdigest()
        # every rank's device weights must be the bytes rank 0 folded (a broken broadcast would otherwise go
        # unnoticed: every rank also builds the same seeded weights itself)
        digests = D.allgather_objects(digest, info)
        ref_digest = hashlib.sha256(np.ascontiguousarray(blob0).tobytes()).hexdigest() if info.is_main else None
        ref_digest = D.broadcast_object(ref_digest, info)
        weights_verified = all(d == ref_digest for d in digests)
        if not weights_verified:
            raise RuntimeError(f"replica weights differ after the broadcast: {digests} vs rank 0 {ref_digest}")
        cpu_note = (f"pinned to {len(share)} NUMA-local CPUs" if pinned else "not pinned") + f", {ncpu} usable"
        log(f"[rank {info.rank}/{info.world} {info.backend}] {a.dtype} pipeline ready in {time.time() - t0:.1f}s; "
            f"arena MB {({b: round(v / 2**20, 1) for b, v in pipe.arena_bytes.items()})}; decode workers {workers}; "
            f"{cpu_note}; weights verified")

        if a.fake_engine:
            images = synthetic_images(16, 7, hw=(96, 128))
            man = None
        else:
            images, man = load_workload(pipe, info, a.images, a.seed, a.dtype)
            # the uploads are the JPEGs the workload was curated on (manifest config.jpeg_quality)
            a.jpeg_quality = int(man.config.get("jpeg_quality", a.jpeg_quality))
        jpegs = [encode_jpeg(im, a.jpeg_quality) for im in images]
        off = (info.rank * 37) % len(jpegs)
        jpegs_r = jpegs[off:] + jpegs[:off]

        from inference_arena_amd.labels import load_labels

        levels = {}
        sec: dict = {}
        R = a.batch * a.step_batches
        if a.path == "http":
            batcher = native().DynamicBatcher([ex], batcher_config(a))
            fe = native().HttpFrontEnd(batcher, pool.native_channel(), list(load_labels(None)),
                                       {"host": "127.0.0.1", "port": 0, "io_threads": a.http_threads})
            reqs = [http_request(j) for j in jpegs_r]
            gc.collect()
            gc.freeze()
            window, lat, crops, status = measure_http(fe.port, reqs, a, info, D, sync, a.users)
            errs = int((status != 200).sum())
            lat = list(lat)
            bs = []
            fe.stop()
            fe = None
            batcher.shutdown()
            if info.is_main and a.latency_levels:
                # the reference's low user levels behind a batcher with a short busy delay (a lone request
                # waits 100 us, a loaded device 500 us for its batch to fill), on the same decode processes
                cfg = dict(batcher_config(a), max_queue_delay_us=a.level_delay_us)
                batcher = native().DynamicBatcher([ex], cfg)
                fe = native().HttpFrontEnd(batcher, pool.native_channel(), list(load_labels(None)),
                                           {"host": "127.0.0.1", "port": 0, "io_threads": a.http_threads})
                levels = latency_levels(fe.port, reqs, [int(u) for u in a.latency_levels.split(",") if u], a)
                levels["batcher"] = {"max_queue_delay_us": cfg["max_queue_delay_us"],
                                     "idle_queue_delay_us": cfg["idle_queue_delay_us"]}
                fe.stop()
                fe = None
                batcher.shutdown()
            D.barrier(info)
            pool.to_python_mode()
            if a.secondary_inproc:
                w2, lat2, _, _, _ = measure_inproc(ex, pool, jpegs, a, info, D, sync)
                w2 = D.allreduce_max(w2, info)
                sec["inproc"] = {"value": round(a.steps * R * info.world / w2, 2),
                                 "p50_ms": round(float(np.percentile(lat2, 50)) * 1e3, 3),
                                 "p99_ms": round(float(np.percentile(lat2, 99)) * 1e3, 3)}
        else:
            window, lat, crops, bs, errs = measure_inproc(ex, pool, jpegs, a, info, D, sync)
        t_max = D.allreduce_max(window, info)
        per_rank = D.allgather_floats([a.steps * R / window], info)

        eng = None
        if not a.fake_engine and a.engine_batches > 0:
            eng = engine_throughput(ex, images, a.batch, a.engine_batches)
        if not a.fake_engine and a.secondary_bf16 and a.dtype != "bf16":
            alt = GpuPipeline(yolo, mnet, device=dev, buckets=buckets, crop_cap_per_image=a.crop_cap, dtype="bf16")
            w2, lat2, _, _, _ = measure_inproc(alt.ex, pool, jpegs, a, info, D, sync)
            w2 = D.allreduce_max(w2, info)
            sec["bf16"] = {"value": round(a.steps * R * info.world / w2, 2),
                           "p50_ms": round(float(np.percentile(lat2, 50)) * 1e3, 3),
                           "p99_ms": round(float(np.percentile(lat2, 99)) * 1e3, 3),
                           "path": "inproc",
                           "engine_req_s": round(engine_throughput(alt.ex, images, a.batch, a.engine_batches), 1)}

        all_lat = D.allgather_floats([float(x) for x in lat], info)
        all_crops = D.allgather_floats([float(c) for c in crops], info)
        all_eng = D.allgather_floats([eng or 0.0], info)
        all_err = D.allgather_floats([float(errs)], info)
        all_cpu = D.allgather_floats([float(len(share)) if pinned else float(ncpu)], info)
        D.barrier(info)
        if info.is_main:
            flat = np.asarray([x for lst in all_lat for x in lst]) * 1e3
            total_req = a.steps * R * info.world
            fan = float(np.sum([x for lst in all_crops for x in lst]) / max(1, len(flat)))
            value = total_req / t_max
            cpu_budget = min(x[0] for x in all_cpu)
            if cpu_budget < value / info.world / 1000.0:
                log(f"warning: {cpu_budget:.0f} CPUs per rank for {value / info.world:.0f} req/s per rank "
                    f"(< 1 core per 1k req/s: host-bound)")
            out = {
                "metric": METRIC,
                "value": round(value, 2),
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
                         "fan-out %.2f); random-init YOLOv5nu + MobileNetV2 weights; per-request end to end%s, "
                         "%d closed-loop users/GPU"
                         % (a.jpeg_quality, fan, " over HTTP: multipart upload -> native front end -> JPEG decode "
                            "-> dynamic batching -> full device pipeline -> JSON response" if a.path == "http" else
                            ": JPEG decode + dynamic batching + full device pipeline + result split", a.users))
                        + ("; FAKE ENGINE (host-only EchoInstance, CPU test)" if a.fake_engine else ""),
                "config": {
                    "model": "YOLOv5nu(640)->MobileNetV2(224)",
                    "global_batch": a.batch * info.world,
                    "seq_len": None,
                    "parallelism": f"dp{info.world}",
                    "per_gpu_batch": a.batch,
                    "requests_per_step_per_gpu": R,
                    "users_per_gpu": a.users,
                    "image_size": 640,
                    "crop_size": 224,
                    "decode_workers_per_gpu": workers,
                    "workload": ({"images": len(images), "distribution": man.distribution,
                                  "mean_detections": man.statistics.get("mean_detections")} if man else
                                 {"images": len(images)}),
                },
                "path": a.path,
                "p50_ms": round(float(np.percentile(flat, 50)), 3),
                "p99_ms": round(float(np.percentile(flat, 99)), 3),
                "latency": ("per-request end to end at the client (upload sent -> JSON response parsed)"
                            if a.path == "http" else "per-request end to end (JPEG bytes in -> results out)"),
                "mean_crops_per_request": round(fan, 3),
                "mean_batch": round(float(np.mean(bs)), 2) if bs else None,
                "errors": int(sum(x for lst in all_err for x in lst)),
                "engine_req_s": round(float(sum(x for lst in all_eng for x in lst)), 1) if eng else None,
                "levels": levels,
                "bs1_p50_ms": (levels.get("1") or {}).get("p50_ms"),
                "bs1_p99_ms": (levels.get("1") or {}).get("p99_ms"),
                "per_rank_req_s": [round(x[0], 1) for x in per_rank],
                "collective_backend": info.backend,
                "weights_verified": bool(weights_verified),
                "cpu_share_per_rank": [int(x[0]) for x in all_cpu],
                "world_size_checked": info.world,
            }
            out.update(sec)
            print(json.dumps(out), flush=True)
    finally:
        if fe is not None:
            fe.stop()
        pool.close()
    D.shutdown(info)
    return 0


if __name__ == "__main__":
    sys.exit(main())
