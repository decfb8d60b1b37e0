"""Python face of the native GPU pipeline (one instance per GPU).

``GpuPipeline`` lowers the two networks into an executor program
(``plans.plan_pipeline``), uploads the weight blob, lays out and captures one
hipGraph per batch bucket and exposes ``infer`` / ``submit``+``collect``.
Results are returned per image as ``ImageResult``: detections in original
image coordinates (reference order: class id asc, score desc) and, for each
detection, the classifier's top-5 (ids, raw logits, softmax probabilities).
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field

import numpy as np

from ..config import get_controlled_variable, get_gpu_config, get_model_config
from ..models.mobilenetv2 import MobileNetV2
from ..models.yolov5nu import YOLOv5nu
from ..ops import native
from .planner import layout
from .plans import (plan_classifier, plan_detector, plan_mobilenet_raw, plan_pipeline, plan_split_classifier,
                    plan_split_detector, plan_yolo_raw)
from .validate import validate_program


@dataclass
class ImageResult:
    boxes: np.ndarray  # [K, 4] x1, y1, x2, y2 (original image coords)
    scores: np.ndarray  # [K]
    classes: np.ndarray  # [K] detector class ids
    topk_idx: np.ndarray  # [K, 5]
    topk_logit: np.ndarray  # [K, 5]
    topk_prob: np.ndarray  # [K, 5]
    det_count: int = 0  # detections kept by NMS (may exceed K when max_det clips)
    timing: dict = field(default_factory=dict)

    def __len__(self) -> int:
        return int(self.boxes.shape[0])


def split_results(res: dict, n: int, gpu_ms: float | None = None) -> list[ImageResult]:
    det = res["det"]
    cnt = res["det_count"]
    offs = res["crop_offset"]
    out = []
    max_det = det.shape[1]
    for i in range(n):
        k = int(min(cnt[i], max_det))
        d = det[i, :k]
        a, b = int(offs[i]), int(offs[i + 1])
        out.append(
            ImageResult(
                boxes=d[:, :4].copy(),
                scores=d[:, 4].copy(),
                classes=d[:, 5].copy().view(np.int32),
                topk_idx=res["topk_idx"][a:b],
                topk_logit=res["topk_logit"][a:b],
                topk_prob=res["topk_prob"][a:b],
                det_count=int(cnt[i]),
                timing={"gpu_ms": float(res.get("gpu_ms", gpu_ms or 0.0)), "batch_bucket": int(res.get("bucket", 0))},
            )
        )
    return out


def resolve_dtype(dtype: str | None = None) -> str:
    """Pipeline precision: the explicit argument, else ``ARENA_DTYPE``, else experiment.yaml ``gpu.dtype``.

    ``fp32`` (default) reproduces the reference's fp32 ONNX Runtime numerics with the exact-fp32 kernels;
    ``bf16`` selects the tuned bf16 kernels (fp32 accumulation)."""
    d = dtype or os.environ.get("ARENA_DTYPE") or str(get_gpu_config().get("dtype", "fp32"))
    d = {"float32": "fp32", "f32": "fp32", "bfloat16": "bf16"}.get(d.lower(), d.lower())
    if d not in ("fp32", "bf16"):
        raise ValueError(f"unsupported pipeline dtype {d!r} (fp32 or bf16)")
    return d


class GpuProgramRunner:
    """One native Executor running one program, with a hipGraph per batch bucket.

    Base of every GPU model object: the fused pipeline (``GpuPipeline``), the
    split detector / classifier programs used by the microservices arm and the
    reference-contract tensor models served by the model server.
    """

    def __init__(self, program, *, device: int = 0, buckets=None, max_det: int | None = None,
                 crop_cap_per_image: int | None = None, host_threads: int | None = None,
                 pool_bytes_per_image: int = 640 * 640 * 3, weights: np.ndarray | None = None,
                 share_buffers: bool = True):
        gcfg = get_gpu_config()
        self.program = program
        self.buckets = sorted(int(b) for b in (buckets or gcfg["batch_buckets"]))
        self.max_det = int(max_det or program.meta.get("max_det") or gcfg["max_det"])
        self.raw_out_bytes = int(program.meta.get("raw_out_bytes", 0))
        C = native()
        self.ex = C.Executor({
            "device": int(device),
            "max_batch": self.buckets[-1],
            "max_det": self.max_det,
            "cand_cap": int(program.meta.get("cand_cap", 8400)),
            "crop_cap_per_image": int(crop_cap_per_image or gcfg["crop_cap_per_image"]),
            "pool_bytes_per_image": int(pool_bytes_per_image),
            "det_size": int(program.meta.get("det_size", 640)),
            "cls_size": int(program.meta.get("cls_size", 224)),
            "host_threads": int(host_threads or gcfg["host_threads"]),
            "raw_out_bytes": self.raw_out_bytes,
        })
        if weights is not None and weights.nbytes != program.weights.nbytes:
            raise ValueError("weight blob does not match the program's layout")
        self.ex.set_weights(program.weights if weights is None else weights)
        self.ex.set_program(program.ops, program.cls_ops)
        self.arena_bytes = {}
        self.offsets = {}
        for B in self.buckets:
            cc = self.ex.crop_cap_for(B)
            validate_program(program, B, cc, max_det=self.max_det, cand_cap=int(program.meta.get("cand_cap", 8400)),
                             raw_out_bytes=self.raw_out_bytes)
            offs, total = layout(program.buffers, B, cc, share=share_buffers)
            self._add_bucket(B, offs, total)
            self.arena_bytes[B] = total
            self.offsets[B] = offs
        self.device = device

    def _add_bucket(self, B: int, offs, total: int) -> None:
        """Capture bucket B with conv kernel choices from the persisted tuning table (engine/tuning.py)."""
        from . import tuning

        ops = self.program.ops
        m = tuning.mode()
        if m == "off" or not tuning.needs_tuning(ops):
            self.ex.add_bucket(B, offs, total, [0] * len(ops) if m == "off" else None)
            self.tuning_source = "off" if m == "off" else "n/a"
            return
        table = tuning.lookup(ops, B) if m == "table" else None
        if table is not None:
            self.ex.add_bucket(B, offs, total, table)
            self.tuning_source = "table"
            return
        self.ex.add_bucket(B, offs, total)  # times every conv family, captures the fastest
        tuning.store(ops, B, self.ex.conv_choices(B))
        self.tuning_source = "tuned"

    @property
    def kind(self) -> str:
        return str(self.program.meta.get("kind", "pipeline"))

    @property
    def dtype(self) -> str:
        return str(self.program.meta.get("dtype", "bf16"))

    def read_buffer(self, name: str, B: int, item: int = 0) -> np.ndarray:
        """Debug: NHWC contents of a planner buffer for one batch item (fp32)."""
        import torch

        buf = next(b for b in self.program.buffers if b.name == name)
        raw = self.ex.read_arena(B, int(self.offsets[B][buf.id]) + item * buf.per_item, buf.H * buf.W * buf.C * buf.elem)
        t = torch.from_numpy(raw.copy())
        t = t.view(torch.bfloat16).float() if buf.elem == 2 else t.view(torch.float32)
        return t.reshape(buf.H, buf.W, buf.C).numpy()

    @property
    def max_batch(self) -> int:
        return self.buckets[-1]

    def run_raw(self, inputs: list[np.ndarray]) -> list[dict]:
        """Run ``inputs`` through the executor in max-batch chunks; raw result dicts."""
        out = []
        for k in range(0, len(inputs), self.max_batch):
            out.append(self.ex.run(list(inputs[k: k + self.max_batch])))
        return out

class GpuPipeline(GpuProgramRunner):
    """The fused detect -> crop -> classify program (monolithic / model-server ensemble)."""

    def __init__(self, yolo: YOLOv5nu, mnet: MobileNetV2, *, device: int = 0, buckets=None, max_det: int | None = None,
                 crop_cap_per_image: int | None = None, host_threads: int | None = None,
                 max_image_pixels: int = 640 * 640, conf_thr: float | None = None, iou_thr: float | None = None,
                 weights: np.ndarray | None = None, share_buffers: bool = True, dtype: str | None = None):
        gcfg = get_gpu_config()
        ycfg = get_model_config("yolov5n")
        mb = get_controlled_variable("preprocessing", "mobilenet")
        det_size = int(get_controlled_variable("preprocessing", "yolo")["target_size"])
        cls_size = int(mb["target_size"])
        self.conf_thr = float(conf_thr if conf_thr is not None else ycfg["confidence_threshold"])
        self.iou_thr = float(iou_thr if iou_thr is not None else ycfg["iou_threshold"])
        max_det = int(max_det or gcfg["max_det"])
        program = plan_pipeline(yolo, mnet, conf_thr=self.conf_thr, iou_thr=self.iou_thr, det_size=det_size,
                                cls_size=cls_size, mean=mb["mean"], std=mb["std"], max_det=max_det,
                                dtype=resolve_dtype(dtype))
        super().__init__(program, device=device, buckets=buckets, max_det=max_det,
                         crop_cap_per_image=crop_cap_per_image, host_threads=host_threads,
                         pool_bytes_per_image=int(max_image_pixels) * 3, weights=weights,
                         share_buffers=share_buffers)

    def submit(self, images: list[np.ndarray]) -> int:
        return self.ex.submit([np.ascontiguousarray(i, dtype=np.uint8) for i in images])

    def collect(self, slot: int, n: int) -> list[ImageResult]:
        return split_results(self.ex.collect(slot), n)

    def infer(self, images: list[np.ndarray]) -> list[ImageResult]:
        out: list[ImageResult] = []
        for k in range(0, len(images), self.max_batch):
            chunk = images[k : k + self.max_batch]
            res = self.ex.run([np.ascontiguousarray(i, dtype=np.uint8) for i in chunk])
            out.extend(split_results(res, len(chunk)))
        return out


class SplitPipeline:
    """Split topology: detection on GPU ``det_device``, classification on GPU ``cls_device``; the crop plan,
    detections and decoded images move device to device (xGMI peer copies, csrc/runtime/split.h) instead of
    the reference's per-crop JPEG + gRPC hop.  Same results as ``GpuPipeline``; ``instance`` is a batch
    instance for the native DynamicBatcher."""

    def __init__(self, yolo: YOLOv5nu, mnet: MobileNetV2, *, det_device: int = 0, cls_device: int = 1,
                 buckets=None, max_det: int | None = None, crop_cap_per_image: int | None = None,
                 conf_thr: float | None = None, iou_thr: float | None = None, dtype: str | None = None,
                 max_image_pixels: int = 640 * 640):
        gcfg = get_gpu_config()
        ycfg = get_model_config("yolov5n")
        mb = get_controlled_variable("preprocessing", "mobilenet")
        det_size = int(get_controlled_variable("preprocessing", "yolo")["target_size"])
        d = resolve_dtype(dtype)
        max_det = int(max_det or gcfg["max_det"])
        conf = float(conf_thr if conf_thr is not None else ycfg["confidence_threshold"])
        iou = float(iou_thr if iou_thr is not None else ycfg["iou_threshold"])
        kw = dict(buckets=buckets, max_det=max_det, crop_cap_per_image=crop_cap_per_image,
                  pool_bytes_per_image=int(max_image_pixels) * 3)
        self.det = GpuProgramRunner(plan_split_detector(yolo, conf_thr=conf, iou_thr=iou, det_size=det_size,
                                                        max_det=max_det, dtype=d), device=det_device, **kw)
        self.cls = GpuProgramRunner(plan_split_classifier(mnet, cls_size=int(mb["target_size"]), mean=mb["mean"],
                                                          std=mb["std"], max_det=max_det, dtype=d),
                                    device=cls_device, **kw)
        self.cls.ex.set_peer_stage(True)
        self.instance = native().SplitInstance(self.det.ex, self.cls.ex)
        self.max_batch = self.det.max_batch
        self.dtype = d

    def submit(self, images: list[np.ndarray]) -> int:
        return self.instance.submit([np.ascontiguousarray(i, dtype=np.uint8) for i in images])

    def collect(self, slot: int, n: int) -> list[ImageResult]:
        return split_results(self.instance.collect(slot), n)

    def infer(self, images: list[np.ndarray]) -> list[ImageResult]:
        out: list[ImageResult] = []
        for k in range(0, len(images), self.max_batch):
            chunk = images[k: k + self.max_batch]
            out.extend(self.collect(self.submit(chunk), len(chunk)))
        return out


class GpuDetector(GpuProgramRunner):
    """Detection-only program (microservices detection service): letterbox -> YOLO -> decode -> NMS."""

    def __init__(self, yolo: YOLOv5nu, *, device: int = 0, buckets=None, conf_thr: float | None = None,
                 iou_thr: float | None = None, max_det: int | None = None, max_image_pixels: int = 640 * 640,
                 dtype: str | None = None, **kw):
        ycfg = get_model_config("yolov5n")
        det_size = int(get_controlled_variable("preprocessing", "yolo")["target_size"])
        self.conf_thr = float(conf_thr if conf_thr is not None else ycfg["confidence_threshold"])
        self.iou_thr = float(iou_thr if iou_thr is not None else ycfg["iou_threshold"])
        max_det = int(max_det or get_gpu_config()["max_det"])
        prog = plan_detector(yolo, conf_thr=self.conf_thr, iou_thr=self.iou_thr, det_size=det_size, max_det=max_det,
                             dtype=resolve_dtype(dtype))
        super().__init__(prog, device=device, buckets=buckets, max_det=max_det,
                         pool_bytes_per_image=int(max_image_pixels) * 3, **kw)

    def infer(self, images: list[np.ndarray]) -> list[ImageResult]:
        imgs = [np.ascontiguousarray(i, dtype=np.uint8) for i in images]
        out: list[ImageResult] = []
        for k, res in enumerate(self.run_raw(imgs)):
            n = min(self.max_batch, len(imgs) - k * self.max_batch)
            out.extend(split_results(res, n))
        return out


class GpuClassifier(GpuProgramRunner):
    """Classification-only program (microservices classification service): every input is one crop,
    resized to 224 and normalised on the device, then MobileNetV2 + top-5 softmax."""

    def __init__(self, mnet: MobileNetV2, *, device: int = 0, buckets=None, max_image_pixels: int = 640 * 640,
                 dtype: str | None = None, **kw):
        mb = get_controlled_variable("preprocessing", "mobilenet")
        prog = plan_classifier(mnet, cls_size=int(mb["target_size"]), mean=mb["mean"], std=mb["std"],
                               dtype=resolve_dtype(dtype))
        super().__init__(prog, device=device, buckets=buckets, pool_bytes_per_image=int(max_image_pixels) * 3, **kw)

    def infer(self, crops: list[np.ndarray]) -> list[tuple[np.ndarray, np.ndarray, np.ndarray]]:
        """Per crop: (top-5 class ids, raw logits, softmax probabilities)."""
        imgs = [np.ascontiguousarray(i, dtype=np.uint8) for i in crops]
        out = []
        for res in self.run_raw(imgs):
            offs = res["crop_offset"]
            for i in range(len(offs) - 1):
                a = int(offs[i])
                out.append((res["topk_idx"][a], res["topk_logit"][a], res["topk_prob"][a]))
        return out


class GpuFrameClassifier(GpuProgramRunner):
    """Crop gather + MobileNetV2 over whole frames already resident in device memory (arm B device
    transport, server/device_transport.py): the second stage of the split topology fed by
    ``Executor.submit_device`` — frames named by device pointer (IPC-mapped from the detection process),
    boxes in original-image pixels — instead of by a peer executor's slot."""

    def __init__(self, mnet: MobileNetV2, *, device: int = 0, buckets=None, max_det: int | None = None,
                 max_image_pixels: int = 640 * 640, dtype: str | None = None, **kw):
        mb = get_controlled_variable("preprocessing", "mobilenet")
        max_det = int(max_det or get_gpu_config()["max_det"])
        prog = plan_split_classifier(mnet, cls_size=int(mb["target_size"]), mean=mb["mean"], std=mb["std"],
                                     max_det=max_det, dtype=resolve_dtype(dtype))
        super().__init__(prog, device=device, buckets=buckets, max_det=max_det,
                         pool_bytes_per_image=int(max_image_pixels) * 3, **kw)
        self.ex.set_peer_stage(True)
        self.max_image_pixels = int(max_image_pixels)

    def submit(self, images, boxes) -> int:
        """``images``: [(device pointer, height, width, device)]; ``boxes``: float32 [k, 6] per image."""
        return self.ex.submit_device(list(images), [np.ascontiguousarray(b, dtype=np.float32) for b in boxes])

    def collect(self, slot: int) -> dict:
        return self.ex.collect(slot)


class GpuTensorModel(GpuProgramRunner):
    """Reference tensor contract models served by the model server:

    * ``yolov5n``: FP32 [3, 640, 640] -> FP32 [84, 8400] (raw detection head)
    * ``mobilenetv2``: FP32 [3, 224, 224] (ImageNet-normalised) -> FP32 [1000] logits
    """

    def __init__(self, program, *, device: int = 0, buckets=None, **kw):
        S = int(program.meta.get("det_size") if program.meta["kind"] == "yolo_raw" else program.meta["cls_size"])
        self.input_shape = (3, S, S)
        self.output_shape = tuple(program.meta["output_shape"])
        super().__init__(program, device=device, buckets=buckets, pool_bytes_per_image=3 * S * S * 4, **kw)

    @classmethod
    def yolo(cls, yolo: YOLOv5nu, dtype: str | None = None, **kw) -> "GpuTensorModel":
        det_size = int(get_controlled_variable("preprocessing", "yolo")["target_size"])
        return cls(plan_yolo_raw(yolo, det_size=det_size, dtype=resolve_dtype(dtype)), **kw)

    @classmethod
    def mobilenet(cls, mnet: MobileNetV2, dtype: str | None = None, **kw) -> "GpuTensorModel":
        cls_size = int(get_controlled_variable("preprocessing", "mobilenet")["target_size"])
        return cls(plan_mobilenet_raw(mnet, cls_size=cls_size, dtype=resolve_dtype(dtype)), **kw)

    def infer(self, tensors) -> np.ndarray:
        """``tensors``: float32 [N, 3, S, S] (or a list of [3, S, S]); returns float32 [N, *output_shape]."""
        xs = [np.ascontiguousarray(t, dtype=np.float32) for t in tensors]
        for x in xs:
            if x.shape != self.input_shape:
                raise ValueError(f"expected input shape {self.input_shape}, got {x.shape}")
        outs = [r["raw"].view(np.float32).reshape(-1, *self.output_shape) for r in self.run_raw(xs)]
        return np.concatenate(outs, 0) if outs else np.zeros((0, *self.output_shape), np.float32)
