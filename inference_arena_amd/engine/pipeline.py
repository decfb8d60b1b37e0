"""Python face of the native GPU pipeline (one instance per GPU).

``GpuPipeline`` lowers the two networks into an executor program
(``plans.plan_pipeline``), uploads the weight blob, lays out and captures one
hipGraph per batch bucket and exposes ``infer`` / ``submit``+``collect``.
Results are returned per image as ``ImageResult``: detections in original
image coordinates (reference order: class id asc, score desc) and, for each
detection, the classifier's top-5 (ids, raw logits, softmax probabilities).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from ..config import get_controlled_variable, get_gpu_config, get_model_config
from ..models.mobilenetv2 import MobileNetV2
from ..models.yolov5nu import YOLOv5nu
from ..ops import native
from .planner import layout
from .plans import plan_pipeline


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


class GpuPipeline:
    def __init__(self, yolo: YOLOv5nu, mnet: MobileNetV2, *, device: int = 0, buckets=None, max_det: int | None = None,
                 crop_cap_per_image: int | None = None, host_threads: int | None = None,
                 max_image_pixels: int = 640 * 640, conf_thr: float | None = None, iou_thr: float | None = None,
                 weights: np.ndarray | None = None, share_buffers: bool = True):
        gcfg = get_gpu_config()
        ycfg = get_model_config("yolov5n")
        mb = get_controlled_variable("preprocessing", "mobilenet")
        det_size = int(get_controlled_variable("preprocessing", "yolo")["target_size"])
        cls_size = int(mb["target_size"])
        self.buckets = sorted(int(b) for b in (buckets or gcfg["batch_buckets"]))
        self.max_det = int(max_det or gcfg["max_det"])
        self.conf_thr = float(conf_thr if conf_thr is not None else ycfg["confidence_threshold"])
        self.iou_thr = float(iou_thr if iou_thr is not None else ycfg["iou_threshold"])
        self.program = plan_pipeline(yolo, mnet, conf_thr=self.conf_thr, iou_thr=self.iou_thr, det_size=det_size,
                                     cls_size=cls_size, mean=mb["mean"], std=mb["std"], max_det=self.max_det)
        C = native()
        self.ex = C.Executor({
            "device": int(device),
            "max_batch": self.buckets[-1],
            "max_det": self.max_det,
            "cand_cap": 8400,
            "crop_cap_per_image": int(crop_cap_per_image or gcfg["crop_cap_per_image"]),
            "pool_bytes_per_image": int(max_image_pixels) * 3,
            "det_size": det_size,
            "cls_size": cls_size,
            "host_threads": int(host_threads or gcfg["host_threads"]),
        })
        if weights is not None and weights.nbytes != self.program.weights.nbytes:
            raise ValueError("weight blob does not match the program's layout")
        self.ex.set_weights(self.program.weights if weights is None else weights)
        self.ex.set_program(self.program.ops, self.program.cls_ops)
        self.arena_bytes = {}
        self.offsets = {}
        for B in self.buckets:
            offs, total = layout(self.program.buffers, B, self.ex.crop_cap_for(B), share=share_buffers)
            self.ex.add_bucket(B, offs, total)
            self.arena_bytes[B] = total
            self.offsets[B] = offs
        self.device = device

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
