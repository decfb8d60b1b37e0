"""Core of the arena model server (the Triton-equivalent of arm C).

Reference: Triton 24.08 serving an ONNX Runtime model repository
(architectures/triton/docker-compose.yml:79-147) with ``max_batch_size: 0``
and the default scheduler (infrastructure/minio/triton_config.py:98-128).

Here every model of the repository is compiled into executor programs
(``platform: "arena_hip"``):

* tensor models keep the reference contract — ``yolov5n``: FP32
  [N,3,640,640] -> ``output0`` [N,84,8400]; ``mobilenetv2``: FP32
  [N,3,224,224] -> ``output`` [N,1000] — running ``GpuTensorModel``
  programs; ``instance_group.count`` executors share one native dynamic
  batcher configured from ``dynamic_batching`` (none -> batch 1, no delay,
  like Triton's default scheduler);
* the ensemble ``arena_pipeline`` (detector -> classifier) is compiled into
  ONE fused device program (``GpuPipeline``) instead of chaining models.

``device="cpu"`` serves the same models with fp32 torch (tests, CPU arm); ``device="fake"`` serves only the
ensemble, on the host-only EchoInstance (CPU tests of the per-GPU process layout).
"""
from __future__ import annotations

import asyncio
import os
import logging
import threading
import time
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass, field

import numpy as np

from ..repository import model_config as mc
from ..repository.store import ARCHS, ModelEntry, load_module, scan_repository
from .batching import AsyncBatcher, TooLarge

log = logging.getLogger("arena.modelserver")


class InferError(Exception):
    """Client error (bad input / unknown model): INVALID_ARGUMENT / 400."""

    def __init__(self, msg: str, code: str = "INVALID_ARGUMENT"):
        super().__init__(msg)
        self.code = code


@dataclass
class ModelStats:
    success: int = 0
    failure: int = 0
    inference_count: int = 0
    execution_count: int = 0
    last_inference_ms: int = 0
    request_us: float = 0.0
    queue_us: float = 0.0
    compute_us: float = 0.0
    lock: threading.Lock = field(default_factory=threading.Lock)

    def record(self, ok: bool, n_items: int, req_us: float, queue_us: float = 0.0, compute_us: float = 0.0):
        with self.lock:
            if ok:
                self.success += 1
                self.inference_count += n_items
                self.execution_count += 1
                self.request_us += req_us
                self.queue_us += queue_us
                self.compute_us += compute_us
            else:
                self.failure += 1
            self.last_inference_ms = int(time.time() * 1e3)


class ModelHandle:
    platform = mc.PLATFORM

    def __init__(self, entry: ModelEntry):
        self.entry = entry
        self.name = entry.name
        self.config = entry.config
        self.version = str(entry.versions[-1]) if entry.versions else "1"
        self.stats = ModelStats()
        self.ready = False

    def metadata(self) -> dict:
        def t(x):
            return {"name": x.name, "datatype": mc.TYPE_TO_KSERVE[mc.data_type_name(x.data_type)],
                    "shape": ([-1] if self.config.max_batch_size > 0 else []) + list(x.dims)}

        return {"name": self.name, "versions": [str(v) for v in self.entry.versions] or ["1"],
                "platform": self.config.platform or self.platform,
                "inputs": [t(x) for x in self.config.input], "outputs": [t(x) for x in self.config.output]}

    async def infer(self, inputs: dict[str, np.ndarray], outputs: list[str] | None = None) -> dict[str, np.ndarray]:
        raise NotImplementedError

    def close(self) -> None:
        pass


class TensorModel(ModelHandle):
    """Reference tensor contract: one FP32 input [N?, 3, S, S] -> one FP32 output."""

    def __init__(self, entry: ModelEntry, device: str, gpu: int = 0):
        super().__init__(entry)
        cfg = entry.config
        self.in_name = cfg.input[0].name
        self.out_name = cfg.output[0].name
        dims = list(cfg.input[0].dims)
        self.item_shape = tuple(int(d) for d in (dims[1:] if cfg.max_batch_size == 0 else dims))
        if len(self.item_shape) != 3 or self.item_shape[0] != 3:
            raise ValueError(f"{self.name}: input dims {dims} are not [N,3,S,S]")
        self.max_batch = max(1, int(cfg.max_batch_size))
        module = load_module(entry.model_file(), entry.name)
        arch = ARCHS.get(entry.name) or entry.metadata.get("arch")
        if arch not in ("yolov5nu", "mobilenetv2"):
            arch = "yolov5nu" if type(module).__name__ == "YOLOv5nu" else "mobilenetv2"
        self.arch = arch
        self.device = device
        if device == "gpu":
            from ..engine.registry import build_session
            from ..parallel.placement import instance_devices

            # Triton semantics: `count` instances on each GPU of the group (all visible GPUs when none listed)
            self.devices = instance_devices(list(cfg.instance_group), default_gpu=gpu)
            buckets = sorted({b for b in (1, 2, 4, 8, 16, 32, self.max_batch) if b <= max(self.max_batch, 1)})
            kind = "yolov5n" if arch == "yolov5nu" else "mobilenetv2"
            self.runners = [build_session(kind, module, module, device=d, buckets=buckets) for d in self.devices]
            db = cfg.dynamic_batching if cfg.HasField("dynamic_batching") else None
            self.batcher = AsyncBatcher(self.runners, max_batch=self.max_batch,
                                        preferred=list(db.preferred_batch_size) if db else None,
                                        max_queue_delay_us=int(db.max_queue_delay_microseconds) if db else 0)
            self.out_item_shape = self.runners[0].output_shape
        else:
            import torch

            self.module = module
            self.pool = ThreadPoolExecutor(max_workers=1, thread_name_prefix=f"cpu-{self.name}")
            with torch.no_grad():
                self.out_item_shape = tuple(module(torch.zeros(1, *self.item_shape)).shape[1:])
        self.ready = True

    def _cpu(self, x: np.ndarray) -> np.ndarray:
        import torch

        with torch.no_grad():
            return self.module(torch.from_numpy(np.array(x, dtype=np.float32))).numpy()

    async def infer(self, inputs, outputs=None):
        if self.in_name not in inputs:
            raise InferError(f"expected input '{self.in_name}' for model '{self.name}'")
        x = inputs[self.in_name]
        if x.dtype != np.float32:
            raise InferError(f"input '{self.in_name}': expected FP32, got {x.dtype}")
        if tuple(x.shape[-3:]) != self.item_shape or x.ndim not in (3, 4):
            raise InferError(f"input '{self.in_name}': unexpected shape {list(x.shape)}, expected "
                             f"[{'N' if self.config.max_batch_size else 1},{','.join(map(str, self.item_shape))}]")
        batch_dim = x.ndim == 4
        xs = x.reshape(-1, *self.item_shape)
        if self.config.max_batch_size > 0 and xs.shape[0] > self.config.max_batch_size:
            raise InferError(f"batch {xs.shape[0]} exceeds max_batch_size {self.config.max_batch_size}")
        t0 = time.perf_counter()
        q = c = 0.0
        if self.device == "gpu":
            ds = await self.batcher.run_many([xs[i] for i in range(xs.shape[0])])
            y = np.stack([d["raw"].view(np.float32).reshape(self.out_item_shape) for d in ds])
            q = sum(d["queue_us"] for d in ds)
            c = sum(d["compute_us"] for d in ds)
        else:
            y = await asyncio.get_running_loop().run_in_executor(self.pool, self._cpu, xs)
        self.stats.record(True, xs.shape[0], (time.perf_counter() - t0) * 1e6, q, c)
        return {self.out_name: y if batch_dim else y[0]}

    def close(self) -> None:
        if self.device == "gpu":
            self.batcher.close()
        else:
            self.pool.shutdown(wait=False)


class PipelineModel(ModelHandle):
    """Ensemble detector -> classifier, compiled into one fused program."""

    platform = mc.ENSEMBLE

    def __init__(self, entry: ModelEntry, models: dict[str, ModelEntry], device: str, gpu: int = 0,
                 decode_threads: int = 8):
        super().__init__(entry)
        steps = list(entry.config.ensemble_scheduling.step)
        if len(steps) != 2:
            raise ValueError(f"{self.name}: expected 2 ensemble steps (detector, classifier)")
        det_e, cls_e = models[steps[0].model_name], models[steps[1].model_name]
        params = {k: v.string_value for k, v in entry.config.parameters.items()}
        if device == "fake":  # host-only stand-in engine (CPU tests of the node layout): no networks to load
            from .app_common import DecodePool
            from .backends import FakeBatchedBackend

            self.device = device
            self.decode_pool = DecodePool(decode_threads)
            self.native_decode = True
            self.backend = FakeBatchedBackend(max_batch=int(params.get("max_batch", 32)),
                                              max_queue_delay_us=int(params.get("max_queue_delay_microseconds", 500)),
                                              overlap=int(os.environ.get("ARENA_BATCH_OVERLAP", "1")))
            self.ready = True
            return
        yolo = load_module(det_e.model_file(), det_e.name)
        mnet = load_module(cls_e.model_file(), cls_e.name)
        self.device = device
        # ARENA_DECODE_PROCS > 0: spawned decode processes with shared-memory delivery (PIL's numpy
        # conversion holds the GIL, so decode threads serialise against the gRPC handlers)
        from .app_common import DecodePool

        self.decode_pool = DecodePool(decode_threads)
        self.native_decode = device == "gpu" and os.environ.get("ARENA_NATIVE_DECODE", "1") != "0"
        if device == "gpu":
            from .backends import GpuBatchedBackend

            from ..parallel.placement import parse_gpu_list

            mb = int(params.get("max_batch", 32))
            # ensemble parameter "gpus" ("0,1" / "0-7") or ARENA_GPUS: one fused pipeline per GPU per instance
            devs = parse_gpu_list(params.get("gpus") or os.environ.get("ARENA_GPUS") or "", default=gpu)
            self.backend = GpuBatchedBackend(yolo, mnet, device=gpu, devices=devs,
                                             instances=int(params.get("instance_count", 1)),
                                             max_batch=mb,
                                             # ARENA_ENSEMBLE_QUEUE_DELAY_US overrides the config's delay
                                             max_queue_delay_us=int(os.environ.get("ARENA_ENSEMBLE_QUEUE_DELAY_US", "0")
                                                                    or params.get("max_queue_delay_microseconds", 500)),
                                             # several model-server processes share a GPU: no batch overlap
                                             # (100 users: 6.75k vs 5.59k req/s, profiles/r5_serving/)
                                             overlap=int(os.environ.get("ARENA_BATCH_OVERLAP", "0")))
        else:
            from .backends import CpuReferenceBackend

            self.backend = CpuReferenceBackend(yolo, mnet, threads=2)
        self.ready = True

    async def infer(self, inputs, outputs=None):
        t0 = time.perf_counter()
        if "IMAGE" in inputs:
            img = inputs["IMAGE"]
            if img.dtype != np.uint8 or img.ndim != 3 or img.shape[2] != 3:
                raise InferError("IMAGE must be UINT8 [H, W, 3]")
        elif "IMAGE_BYTES" in inputs:
            raw = inputs["IMAGE_BYTES"].ravel()
            if raw.size != 1:
                raise InferError("IMAGE_BYTES must hold exactly one encoded image")
            img = None
            if self.native_decode:
                # split decoder: Huffman on C++ threads, reconstruction on the GPU inside the batch (PIL only for
                # formats it does not cover); ARENA_NATIVE_DECODE=0 keeps every upload on the PIL pool
                try:
                    res, timing = await self.backend.infer_bytes(bytes(raw[0]), self.decode_pool.decode)
                except (ValueError, TooLarge) as e:
                    raise InferError(str(e)) from e
            else:
                try:
                    img = await self.decode_pool.decode(bytes(raw[0]))
                except Exception as e:
                    raise InferError(str(e)) from e
        else:
            raise InferError("expected input IMAGE or IMAGE_BYTES")
        if img is not None:
            res, timing = await self.backend.infer(img)
        det = np.concatenate([res.boxes, res.scores[:, None], res.classes[:, None].astype(np.float32)], 1) \
            if len(res) else np.zeros((0, 6), np.float32)
        self.stats.record(True, 1, (time.perf_counter() - t0) * 1e6, timing.get("queue_ms", 0) * 1e3,
                          timing.get("gpu_ms", 0) * 1e3)
        k = len(res)
        # [detection_ms, classification_ms, queue_ms, gpu_ms] of this request's batch (device stage times from
        # the program's wall-clock stamps): the gateway's timing keys without a second clock
        stage = np.asarray([timing.get("detection_ms", 0.0), timing.get("classification_ms", 0.0),
                            timing.get("queue_ms", 0.0), timing.get("gpu_ms", 0.0)], np.float32)
        return {"DETECTIONS": det.astype(np.float32), "STAGE_MS": stage,
                "CLASS_IDS": res.topk_idx[:k].astype(np.int32).reshape(k, 5),
                "CLASS_LOGITS": res.topk_logit[:k].astype(np.float32).reshape(k, 5),
                "CLASS_PROBS": res.topk_prob[:k].astype(np.float32).reshape(k, 5)}

    def close(self) -> None:
        self.backend.close()
        self.decode_pool.close()


class ModelServer:
    """Loads every model of a repository; KServe-v2 front-ends call into it."""

    name = "arena-modelserver"
    version = "2.0.0"
    extensions = ["model_repository", "statistics", "binary_tensor_data", "classification_pipeline"]

    def __init__(self, repo_root, *, device: str = "gpu", gpu: int = 0, models: list[str] | None = None):
        self.repo_root = repo_root
        self.device = device
        self.gpu = gpu
        self.entries = scan_repository(repo_root)
        self.models: dict[str, ModelHandle] = {}
        self.failed: dict[str, str] = {}
        wanted = models or list(self.entries)
        if device == "fake":  # the fake engine stands in for the fused ensemble only
            wanted = [n for n in wanted if self.entries[n].config.platform == mc.ENSEMBLE]
        for name in [n for n in wanted if self.entries[n].config.platform != mc.ENSEMBLE] + \
                    [n for n in wanted if self.entries[n].config.platform == mc.ENSEMBLE]:
            e = self.entries[name]
            errs = mc.validate(e.config)
            try:
                if errs:
                    raise ValueError("; ".join(errs))
                if e.config.platform == mc.ENSEMBLE:
                    self.models[name] = PipelineModel(e, self.entries, device, gpu)
                else:
                    self.models[name] = TensorModel(e, device, gpu)
                log.info(f"loaded model {name}")
            except Exception as ex:  # a broken model does not take the server down (Triton behaviour)
                self.failed[name] = str(ex)
                log.error(f"failed to load model {name}: {ex}")
        self.started = time.time()

    def live(self) -> bool:
        return True

    def ready(self) -> bool:
        return bool(self.models) and all(m.ready for m in self.models.values())

    def get(self, name: str, version: str = "") -> ModelHandle:
        m = self.models.get(name)
        if m is None:
            raise InferError(f"Request for unknown model: '{name}' is not found", code="NOT_FOUND")
        if version and version not in (m.version, *map(str, m.entry.versions)):
            raise InferError(f"Request for unknown model: '{name}' version {version} is not found",
                             code="NOT_FOUND")
        return m

    def index(self) -> list[dict]:
        out = []
        for name, e in self.entries.items():
            state = "READY" if name in self.models else "UNAVAILABLE"
            out.append({"name": name, "version": str(e.versions[-1]) if e.versions else "1", "state": state,
                        "reason": self.failed.get(name, "")})
        return out

    async def infer(self, name: str, inputs: dict[str, np.ndarray], outputs: list[str] | None = None,
                    version: str = "") -> dict[str, np.ndarray]:
        m = self.get(name, version)
        t0 = time.perf_counter()
        try:
            res = await m.infer(inputs, outputs)
        except InferError:
            m.stats.record(False, 0, (time.perf_counter() - t0) * 1e6)
            raise
        except Exception:
            m.stats.record(False, 0, (time.perf_counter() - t0) * 1e6)
            raise
        if outputs:
            missing = [o for o in outputs if o not in res]
            if missing:
                raise InferError(f"unknown output(s) {missing} for model '{name}'")
            res = {k: res[k] for k in outputs}
        return res

    def close(self) -> None:
        for m in self.models.values():
            m.close()
