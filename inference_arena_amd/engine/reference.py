"""fp32 PyTorch/NumPy reference of the full request pipeline.

This is the monolithic arm's algorithm (architectures/monolithic/app/
inference.py:127-227) executed with the torch oracles instead of ONNX Runtime:
letterbox -> YOLOv5nu -> parse_yolo_output (NMS) -> scale_boxes -> per
detection extract_crop -> MobileNet preprocess -> MobileNetV2 -> top-5.
It is the CPU arm of the arena and the end-to-end oracle of GpuPipeline.
"""
from __future__ import annotations

import copy

import numpy as np
import torch

from ..models.mobilenetv2 import MobileNetV2
from ..models.yolov5nu import YOLOv5nu
from ..postprocess import parse_yolo_output
from ..processing import MobileNetPreprocessor, YOLOPreprocessor, extract_crop
from .pipeline import ImageResult


class ReferencePipeline:
    def __init__(self, yolo: YOLOv5nu, mnet: MobileNetV2, conf_thr: float = 0.5, iou_thr: float = 0.45,
                 device: str | torch.device = "cpu", max_det: int | None = None):
        self.yolo = copy.deepcopy(yolo).to(device).eval()
        self.mnet = copy.deepcopy(mnet).to(device).eval()
        self.device = torch.device(device)
        self.conf_thr, self.iou_thr = conf_thr, iou_thr
        self.max_det = max_det
        self.ypre = YOLOPreprocessor()
        self.mpre = MobileNetPreprocessor()

    @torch.no_grad()
    def detect(self, image: np.ndarray) -> np.ndarray:
        r = self.ypre(image)
        out = self.yolo(torch.from_numpy(r.tensor).to(self.device)).float().cpu().numpy()
        det = parse_yolo_output(out, self.conf_thr, self.iou_thr)
        if self.max_det is not None:
            det = det[: self.max_det]
        return r.scale_boxes_to_original(det) if len(det) else det

    @torch.no_grad()
    def classify(self, crops: list[np.ndarray]) -> np.ndarray:
        if not crops:
            return np.zeros((0, 1000), np.float32)
        x = torch.from_numpy(self.mpre.preprocess_batch(crops)).to(self.device)
        return self.mnet(x).float().cpu().numpy()

    def __call__(self, image: np.ndarray) -> ImageResult:
        det = self.detect(image)
        logits = self.classify([extract_crop(image, d) for d in det])
        k = len(det)
        order = np.argsort(-logits, axis=1, kind="stable")[:, :5] if k else np.zeros((0, 5), np.int64)
        top_logit = np.take_along_axis(logits, order, 1) if k else np.zeros((0, 5), np.float32)
        if k:
            z = logits - logits.max(1, keepdims=True)
            p = np.exp(z)
            p /= p.sum(1, keepdims=True)
            top_prob = np.take_along_axis(p, order, 1)
        else:
            top_prob = np.zeros((0, 5), np.float32)
        return ImageResult(
            boxes=det[:, :4].astype(np.float32) if k else np.zeros((0, 4), np.float32),
            scores=det[:, 4].astype(np.float32) if k else np.zeros((0,), np.float32),
            classes=det[:, 5].astype(np.int32) if k else np.zeros((0,), np.int32),
            topk_idx=order.astype(np.int32),
            topk_logit=top_logit.astype(np.float32),
            topk_prob=top_prob.astype(np.float32),
            det_count=k,
        )
