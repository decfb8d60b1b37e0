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
    HTTP + multipart parse -> split JPEG decode (native C++ threads: marker parse + Huffman decode into a
    pinned buffer, csrc/runtime/jpeg_decode.h; PIL processes only for formats it does not cover) -> native
    dynamic batcher (max_batch 32, zero-copy) -> H2D of the coefficients -> GPU dequant + IDCT + chroma
    upsampling + YCbCr->RGB (csrc/kernels/jpeg_idct.hip, bit-exact with PIL) -> letterbox -> YOLOv5nu ->
    decode -> NMS -> crop gather -> MobileNetV2 -> top-5 -> D2H -> JSON response (the reference's schema)
    -> client.
  ``--path inproc`` measures the same pipeline without the HTTP layer (uploads handed to the front end's
  decode stage in process by a C++ closed loop, HttpFrontEnd::submit_local; the JSON is still built); it is
  also reported as the secondary key ``inproc``.
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
pre-decoded images), ``bf16`` (the same HTTP measurement on the bf16 kernels: the host ceiling),
``levels`` (1/10/100 users), ``per_rank_req_s``, ``usable_cpus_per_rank`` (pinned share capped by the job's
cgroup quota divided between the ranks), ``host_cpu_us_per_req`` (host CPU per request by thread class:
HTTP I/O, decode, batcher + JSON, load generator, ...; ``stage_cpu_us_per_req``: HTTP parse, entropy decode,
JSON from thread CPU clocks), ``mean_batch``, ``shared_front`` (N > 1: every rank on one SO_REUSEPORT port
driven by one node-level load generator; ``--front shared`` makes that the headline).

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


def engine_throughput(ex, images, B: int, batches: int, jpeg_set=None) -> float:
    """Device pipeline alone, pipelined submit/collect from one host thread: requests/s between the completion of
    the first ``depth`` batches and the last one (fill and drain excluded).

    ``jpeg_set`` (native ``JpegSet``: the workload's uploads entropy-decoded once into pinned buffers): every batch
    carries the inputs the HTTP path gives the executor — coefficient blocks DMA'd from pinned memory, GPU
    dequantisation / IDCT / colour conversion, then the program — without the per-request Huffman decode, HTTP
    or JSON work; this is the device ceiling of the headline path (``engine_req_s``).  Without it: pre-decoded RGB
    frames, which the executor packs into its pinned staging on the host first (``engine_rgb_req_s``)."""
    depth = ex.num_slots()
    n = len(jpeg_set) if jpeg_set is not None else len(images)
    q, done_t = [], []
    k = 0
    for st in range(batches + depth):
        idx = [(k + i) % n for i in range(B)]
        q.append(ex.submit_jpeg_set(jpeg_set, idx) if jpeg_set is not None else ex.submit([images[i] for i in idx]))
        k += B
        if len(q) == depth:
            ex.collect(q.pop(0))
            done_t.append(time.perf_counter())
    while q:
        ex.collect(q.pop(0))
        done_t.append(time.perf_counter())
    return (len(done_t) - depth) * B / (done_t[-1] - done_t[depth - 1])


def _window(a, info, D, sync, completed, wait_until, users: int, on_open=None):
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
        if on_open is not None:
            on_open()
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


def _thread_cpu() -> dict[str, float]:
    """CPU seconds (user + system) of this process's threads, summed by thread name (native threads name
    themselves: arena-http-io, arena-jpeg, arena-batcher, arena-pack, arena-loadgen, arena-collect)."""
    out: dict[str, float] = {}
    tick = os.sysconf("SC_CLK_TCK")
    for d in Path("/proc/self/task").iterdir():
        try:
            stat = (d / "stat").read_text()
        except OSError:
            continue
        name = stat[stat.index("(") + 1:stat.rindex(")")]
        f = stat[stat.rindex(")") + 2:].split()
        out[name] = out.get(name, 0.0) + (int(f[11]) + int(f[12])) / tick
    return out


def _children_cpu() -> float:
    t = os.times()
    return t.children_user + t.children_system


def torch_device() -> int:
    import torch

    return int(torch.cuda.current_device())


class HostCpu:
    """Host CPU per request over a window, by thread class (+ the decode-pool child processes)."""

    GROUPS = {"arena-http-io": "http_io", "arena-jpeg": "decode", "arena-batcher": "batcher_json",
              "arena-pack": "pack", "arena-loadgen": "loadgen", "arena-collect": "pil_collect"}

    def __init__(self, fe=None):
        self.fe = fe
        self.t0, self.c0 = _thread_cpu(), _children_cpu()
        self.s0 = fe.stats() if fe is not None else None

    def per_request(self, n: int) -> tuple[dict, dict]:
        t1, c1 = _thread_cpu(), _children_cpu()
        by: dict[str, float] = {}
        for name, v in t1.items():
            g = self.GROUPS.get(name, "other")
            by[g] = by.get(g, 0.0) + v - self.t0.get(name, 0.0)
        by["pil_procs"] = c1 - self.c0
        us = {k: round(v / max(1, n) * 1e6, 1) for k, v in sorted(by.items())}
        us["total"] = round(sum(by.values()) / max(1, n) * 1e6, 1)
        stages = {}
        if self.fe is not None:
            s1 = self.fe.stats()
            for k, key in (("http_parse", "cpu_parse_ms"), ("entropy_decode", "cpu_decode_ms"), ("json", "cpu_json_ms")):
                stages[k] = round((s1[key] - self.s0[key]) / max(1, n) * 1e3, 2)
            stages["native_decoded"] = s1["native_decoded"] - self.s0["native_decoded"]
            stages["fallback_decoded"] = s1["fallback_decoded"] - self.s0["fallback_decoded"]
        return us, stages


def _batch_mean(b0: dict, b1: dict) -> float | None:
    """Mean executed batch size between two batcher stats snapshots."""
    nb = b1["batches"] - b0["batches"]
    return round((b1["requests"] - b0["requests"]) / nb, 2) if nb > 0 else None


def measure_http(port: int, reqs: list[bytes], a, info, D, sync, users: int, threads: int, fe=None, batcher=None):
    """Closed-loop HTTP window on one rank: (seconds, latencies s, detections, statuses, extras)."""
    from inference_arena_amd.ops import native

    lg = native().HttpLoadGen({"host": "127.0.0.1", "port": port, "users": users,
                               "threads": max(1, min(threads, users))}, reqs)
    return _measure(lg, a, info, D, sync, users, fe, batcher)


def measure_inproc(fe, uploads: list[bytes], a, info, D, sync, users: int, batcher=None):
    """The same window without the HTTP layer: a C++ closed loop submits the uploads to the front end's decode
    stage in process (HttpFrontEnd::submit_local); decode, batching, device, JSON unchanged."""
    from inference_arena_amd.ops import native

    lg = native().LocalLoadGen(fe, uploads, users)
    return _measure(lg, a, info, D, sync, users, fe, batcher)


def _measure(lg, a, info, D, sync, users, fe, batcher):
    lg.start()

    def wait_until(n):
        if not lg.wait_completed(n, 600.0):
            extra = f" ({lg.connect_failures()} failed connects)" if hasattr(lg, "connect_failures") else ""
            raise TimeoutError(f"load generator: {lg.completed()}/{n} responses{extra}")
    cpu = {}
    try:
        holder = {}

        def opened():
            holder["cpu"] = HostCpu(fe)
            holder["b0"] = batcher.stats() if batcher is not None else None
            if not a.fake_engine:  # device busy over the timed window, 20 Hz (metrics/gpu.py BusySampler)
                # (local query only: ``D`` is the solo stand-in in the node-wide shared-front window)
                from inference_arena_amd.metrics.gpu import BusySampler
                from inference_arena_amd.parallel.dist import device_identity

                try:
                    ident = device_identity(torch_device(), info.rank)
                    holder["busy"] = BusySampler(ident.get("pci_bus_id"), torch_device()).start()
                except Exception as e:  # noqa: BLE001 - a missing sampler must not fail the measurement
                    log(f"gpu busy sampler unavailable: {e}")
        window, c0 = _window(a, info, D, sync, lg.completed, wait_until, users, on_open=opened)
        busy = holder["busy"].stop() if "busy" in holder else None
        n = a.steps * a.batch * a.step_batches
        us, stages = holder["cpu"].per_request(n)
        cpu = {"host_cpu_us_per_req": us, "stage_cpu_us_per_req": stages}
        if busy is not None:
            cpu["gpu_busy"] = busy
        if batcher is not None:
            cpu["mean_batch"] = _batch_mean(holder["b0"], batcher.stats())
    finally:
        lg.stop(60.0)
    r = lg.records(c0, c0 + a.steps * a.batch * a.step_batches)
    return (window, r["latency"].astype(np.float64), r["dets"].astype(np.int64), r["status"].astype(np.int64), cpu)


def latency_levels(port: int, reqs: list[bytes], levels: list[int], a) -> dict:
    """P50/P99/req/s at the reference's closed-loop user levels (one rank's front end, short phases)."""
    from inference_arena_amd.ops import native

    out = {}
    for u in levels:
        log(f"level {u} users")
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


def make_front(batcher, pool, plan: dict, a, port: int = 0, reuse_port: bool = True, jpeg_device: bool = True):
    from inference_arena_amd.labels import load_labels
    from inference_arena_amd.ops import native
    from inference_arena_amd.processing.transforms import max_image_pixels

    return native().HttpFrontEnd(batcher, pool.native_channel(), list(load_labels(None)),
                                 {"host": "127.0.0.1", "port": port, "io_threads": plan["http_io"],
                                  "decode_threads": plan["decode_threads"], "jpeg_device": jpeg_device,
                                  "max_image_pixels": max_image_pixels(), "reuse_port": reuse_port})


def summarize(window: float, lat, a, info, D) -> dict:
    w = D.allreduce_max(window, info)
    flat = np.asarray([x for lst in D.allgather_floats([float(x) for x in lat], info) for x in lst]) * 1e3
    return {"value": round(a.steps * a.batch * a.step_batches * info.world / w, 2),
            "p50_ms": round(float(np.percentile(flat, 50)), 3), "p99_ms": round(float(np.percentile(flat, 99)), 3)}


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
    ap.add_argument("--front", default="per-rank", choices=["per-rank", "shared"],
                    help="per-rank: one port + load generator per rank, value = sum (headline); shared: all ranks "
                         "on one SO_REUSEPORT port driven by one node-level load generator on rank 0")
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--decode-threads", type=int, default=0, help="native split-decoder threads per rank (0: plan)")
    ap.add_argument("--decode-workers", type=int, default=0,
                    help="PIL decode processes per rank (fallback for uploads the split decoder leaves; 0: plan)")
    ap.add_argument("--host-decode", action="store_true",
                    help="reconstruct on the host decode threads instead of the GPU (A/B of the split decoder)")
    ap.add_argument("--http-threads", type=int, default=0, help="epoll I/O threads of the native front end (0: plan)")
    ap.add_argument("--lg-threads", type=int, default=0, help="load-generator threads per rank (0: plan)")
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
                    help="also measure the bf16 kernels over HTTP (secondary key 'bf16': the host ceiling)")
    ap.add_argument("--secondary-shared-front", action=argparse.BooleanOptionalAction, default=True,
                    help="N > 1: also measure one node-level front door (secondary key 'shared_front')")
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
    # are spawned after the pin and inherit it.  The usable count is that share capped by the job's cgroup
    # quota divided between the node's ranks (every rank sees the whole quota).
    from inference_arena_amd.parallel.affinity import host_thread_plan, pin, rank_cpu_share, usable_cpus_per_rank

    share = rank_cpu_share(local_rank, local_world) if not a.fake_engine else None
    pinned = pin(share)
    usable = usable_cpus_per_rank(share if pinned else None, local_world)
    plan = host_thread_plan(usable)
    for key, arg in (("http_io", a.http_threads), ("decode_threads", a.decode_threads),
                     ("loadgen", a.lg_threads), ("pil_procs", a.decode_workers)):
        if arg:
            plan[key] = arg
    budget_warning = None
    if usable < 4:
        budget_warning = (f"rank {local_rank}: only {usable} usable CPUs (pinned share {len(share) if share else '-'}, "
                          f"job quota split {local_world} ways): the host path will bound this rank")
        log("!" * 20 + " " + budget_warning + " " + "!" * 20)
    from inference_arena_amd.server.decode_pool import ProcessDecodePool, prestart

    prestart()
    pool = ProcessDecodePool(workers=plan["pil_procs"], slots=64, native=True, cpus=share if pinned else None)

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

    fronts = []
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
        # which physical GPU each rank drove: N distinct PCI bus ids for an N-GPU record
        rank_devices = D.allgather_objects(D.device_identity(None if a.fake_engine else dev, info.rank,
                                                             a.fake_engine), info)
        shared_gpu = os.environ.get("ARENA_SHARED_GPU") == "1"
        D.check_distinct_devices(rank_devices, shared_gpu)
        torch_world = None
        if not a.fake_engine or info.world > 1:
            import torch.distributed as tdist

            torch_world = tdist.get_world_size() if tdist.is_available() and tdist.is_initialized() else 1
        if torch_world is not None and torch_world != info.world:
            raise RuntimeError(f"torch.distributed world size {torch_world} != WORLD_SIZE {info.world}")
        cpu_note = (f"pinned to {len(share)} NUMA-local CPUs" if pinned else "not pinned") + f", {usable} usable"
        log(f"[rank {info.rank}/{info.world} {info.backend}] {a.dtype} pipeline ready in {time.time() - t0:.1f}s; "
            f"arena MB {({b: round(v / 2**20, 1) for b, v in pipe.arena_bytes.items()})}; host plan {plan}; "
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
        reqs = [http_request(j) for j in jpegs_r]
        jpeg_device = not (a.fake_engine or a.host_decode)

        levels = {}
        sec: dict = {}
        extras: dict = {}
        R = a.batch * a.step_batches

        def serve(engine, cfg=None, port=0, reuse=True):
            b = native().DynamicBatcher([engine], cfg or batcher_config(a))
            f = make_front(b, pool, plan, a, port=port, reuse_port=reuse, jpeg_device=jpeg_device)
            fronts.append((f, b))
            return f, b

        def close(f, b):
            f.stop()
            b.shutdown()
            fronts.remove((f, b))

        # one front end at a time: they share the PIL fallback pool's pipes (one DecodeChannel, one reader)
        gc.collect()
        gc.freeze()
        headline_shared = a.front == "shared" and info.world > 1
        errs = 0
        if not headline_shared:
            fe, batcher = serve(ex)
            if a.path == "http":
                window, lat, crops, status, extras = measure_http(fe.port, reqs, a, info, D, sync, a.users,
                                                                  plan["loadgen"], fe, batcher)
            else:
                window, lat, crops, status, extras = measure_inproc(fe, jpegs_r, a, info, D, sync, a.users, batcher)
            close(fe, batcher)
            errs = int((status != 200).sum())
            lat = list(lat)
            log(f"[rank {info.rank}] headline window: {a.steps * R / window:.0f} req/s")
        if a.path == "http" and info.is_main and a.latency_levels:
            # the reference's low user levels behind a batcher with a short busy delay: a request that finds the
            # device idle is dispatched at once (the reference runs every request alone), a loaded device waits
            # up to 500 us for its batch to fill
            cfg = dict(batcher_config(a), max_queue_delay_us=a.level_delay_us, idle_queue_delay_us=0)
            f2, b2 = serve(ex, cfg)
            levels = latency_levels(f2.port, reqs, [int(u) for u in a.latency_levels.split(",") if u], a)
            log(f"[rank {info.rank}] latency levels: {levels}")
            levels["batcher"] = {"max_queue_delay_us": cfg["max_queue_delay_us"],
                                 "idle_queue_delay_us": cfg["idle_queue_delay_us"]}
            close(f2, b2)
        D.barrier(info)
        if a.path == "http" and a.secondary_inproc and not headline_shared:
            f5, b5 = serve(ex)
            w2, lat2, _, st2, _ = measure_inproc(f5, jpegs_r, a, info, D, sync, a.users, b5)
            close(f5, b5)
            sec["inproc"] = dict(summarize(w2, lat2, a, info, D), errors=int((st2 != 200).sum()))
        if info.world > 1 and (a.secondary_shared_front or headline_shared):
            # one node-level front door: every rank listens on the same port (SO_REUSEPORT spreads the
            # connections), one load generator on rank 0 drives users x world connections
            import socket

            port = 0
            if info.is_main:
                with socket.socket() as sk:
                    sk.bind(("127.0.0.1", 0))
                    port = sk.getsockname()[1]
            port = D.broadcast_object(port, info)
            f3, b3 = serve(ex, port=port)
            D.barrier(info)
            res = None
            if info.is_main:
                # world x the per-rank step: the same requests per GPU as the per-rank windows
                a_node = argparse.Namespace(**vars(a))
                a_node.step_batches = a.step_batches * info.world
                res = measure_http(port, reqs, a_node, _Solo(), _SoloD(), sync, a.users * info.world,
                                   plan["loadgen"] * 2, f3, b3)
            D.barrier(info)
            close(f3, b3)
            if info.is_main:
                w3, lat3, crops3, st3, ex3 = res
                shared = {"value": round(a.steps * R * info.world / w3, 2),
                          "p50_ms": round(float(np.percentile(lat3, 50)) * 1e3, 3),
                          "p99_ms": round(float(np.percentile(lat3, 99)) * 1e3, 3), "errors": int((st3 != 200).sum()),
                          "users": a.users * info.world, "ports": 1, "mean_batch": ex3.get("mean_batch")}
                sec["shared_front"] = shared
                if headline_shared:
                    window, lat, crops, extras = w3, list(lat3), crops3, ex3
                    errs = shared["errors"]
            if headline_shared:
                window = D.broadcast_object(window if info.is_main else None, info)
                if not info.is_main:
                    lat, crops = [], np.zeros(0)
        t_max = D.allreduce_max(window, info)
        per_rank = D.allgather_floats([a.steps * R / window], info)

        eng = eng_rgb = None
        jset = None
        if not a.fake_engine and a.engine_batches > 0:
            jset = native().JpegSet(jpegs_r, pinned=True)
            eng = engine_throughput(ex, images, a.batch, a.engine_batches, jset)
            eng_rgb = engine_throughput(ex, images, a.batch, a.engine_batches)
        if not a.fake_engine and a.secondary_bf16 and a.dtype != "bf16":
            alt = GpuPipeline(yolo, mnet, device=dev, buckets=buckets, crop_cap_per_image=a.crop_cap, dtype="bf16")
            f4, b4 = serve(alt.ex)
            if a.path == "http":
                w4, lat4, _, st4, ex4 = measure_http(f4.port, reqs, a, info, D, sync, a.users, plan["loadgen"], f4, b4)
            else:
                w4, lat4, _, st4, ex4 = measure_inproc(f4, jpegs_r, a, info, D, sync, a.users, b4)
            close(f4, b4)
            sec["bf16"] = dict(summarize(w4, lat4, a, info, D), path=a.path, errors=int((st4 != 200).sum()),
                               mean_batch=ex4.get("mean_batch"), host_cpu_us_per_req=ex4.get("host_cpu_us_per_req"),
                               engine_req_s=round(engine_throughput(alt.ex, images, a.batch, a.engine_batches, jset), 1)
                               if jset is not None else None)

        all_lat = D.allgather_floats([float(x) for x in lat], info)
        all_crops = D.allgather_floats([float(c) for c in crops], info)
        all_eng = D.allgather_floats([eng or 0.0], info)
        all_eng_rgb = D.allgather_floats([eng_rgb or 0.0], info)
        all_err = D.allgather_floats([float(errs)], info)
        all_cpu = D.allgather_floats([float(usable)], info)
        all_ext = D.allgather_objects(extras, info)
        D.barrier(info)
        if info.is_main:
            flat = np.asarray([x for lst in all_lat for x in lst]) * 1e3
            total_req = a.steps * R * info.world
            fan = float(np.sum([x for lst in all_crops for x in lst]) / max(1, len(flat)))
            value = total_req / t_max
            cpu_budget = min(x[0] for x in all_cpu)
            if cpu_budget < value / info.world / 1500.0:
                log(f"warning: {cpu_budget:.0f} usable CPUs per rank for {value / info.world:.0f} req/s per rank "
                    f"(< 1 core per 1.5k req/s: host-bound)")
            ext0 = all_ext[0] or {}
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
                         % (a.jpeg_quality, fan, " over HTTP: multipart upload -> native front end -> split JPEG "
                            "decode (host Huffman, GPU IDCT/colour) -> dynamic batching -> full device pipeline -> "
                            "JSON response" if a.path == "http" else
                            " in process: split JPEG decode + dynamic batching + full device pipeline + JSON", a.users))
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
                    "host_plan_per_gpu": plan,
                    "jpeg_decode": "host" if not jpeg_device else "split: host Huffman + GPU reconstruction",
                    "workload": ({"images": len(images), "distribution": man.distribution,
                                  "mean_detections": man.statistics.get("mean_detections")} if man else
                                 {"images": len(images)}),
                },
                "path": a.path,
                "front": "shared" if headline_shared else "per-rank",
                "p50_ms": round(float(np.percentile(flat, 50)), 3),
                "p99_ms": round(float(np.percentile(flat, 99)), 3),
                "latency": ("per-request end to end at the client (upload sent -> JSON response parsed)"
                            if a.path == "http" else "per-request end to end (upload in -> JSON out, in process)"),
                "mean_crops_per_request": round(fan, 3),
                "mean_batch": ext0.get("mean_batch"),
                "errors": int(sum(x for lst in all_err for x in lst)),
                # device ceiling of the headline path: pre-entropy-decoded JPEG coefficients from pinned memory ->
                # GPU reconstruction -> program (engine_throughput); engine_rgb_req_s: RGB frames packed on the host
                "engine_req_s": round(float(sum(x for lst in all_eng for x in lst)), 1) if eng else None,
                "engine_input": "jpeg coefficients (pinned), GPU reconstruction" if eng else None,
                "engine_rgb_req_s": round(float(sum(x for lst in all_eng_rgb for x in lst)), 1) if eng_rgb else None,
                "levels": levels,
                "bs1_p50_ms": (levels.get("1") or {}).get("p50_ms"),
                "bs1_p99_ms": (levels.get("1") or {}).get("p99_ms"),
                "per_rank_req_s": [round(x[0], 1) for x in per_rank],
                "collective_backend": info.backend,
                "weights_verified": bool(weights_verified),
                "usable_cpus_per_rank": [int(x[0]) for x in all_cpu],
                "cpu_budget_warning": budget_warning,
                "host_cpu_us_per_req": ext0.get("host_cpu_us_per_req"),
                # device busy percent over each rank's timed window, sampled at 20 Hz (amdsmi gfx_activity)
                "gpu_busy": [(x or {}).get("gpu_busy") for x in all_ext] if any(x and x.get("gpu_busy") for x in all_ext)
                else None,
                "stage_cpu_us_per_req": ext0.get("stage_cpu_us_per_req"),
                "world_size_checked": info.world,
                "torch_world_size": torch_world,
                "rank_devices": rank_devices,
                "distinct_gpus": len({d["pci_bus_id"] for d in rank_devices}),
                "shared_gpu_rehearsal": shared_gpu,
            }
            out.update(sec)
            print(json.dumps(out), flush=True)
    finally:
        for f, b in list(fronts):
            f.stop()
            b.shutdown()
        pool.close()
    D.shutdown(info)
    return 0


class _Solo:
    """A one-rank view for rank 0's node-level load generator (the other ranks wait at a barrier)."""
    world, rank, is_main = 1, 0, True


class _SoloD:
    @staticmethod
    def barrier(info):
        pass


if __name__ == "__main__":
    sys.exit(main())
