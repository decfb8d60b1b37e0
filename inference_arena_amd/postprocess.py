"""Detector output post-processing on the host (reference semantics).

``parse_yolo_output`` / ``apply_nms`` follow
architectures/monolithic/app/postprocess.py:12-160 of the reference (identical
copies live in the microservices detection service and the Triton gateway):
[1, 84, N] -> transpose -> max/argmax over the 80 class scores -> keep
conf >= thr -> per-class greedy NMS (suppress IoU > thr, eps 1e-6) ->
[K, 6] = x1, y1, x2, y2, conf, class, ordered by class id then score.

The GPU pipeline runs the same algorithm in csrc/kernels/detect.hip; this
module is its oracle and the CPU arm's implementation.  The inner loop is
vectorised per class instead of the reference's pure-Python while loop, with
identical results.
"""
from __future__ import annotations

import numpy as np


def apply_nms(
    boxes: np.ndarray,
    scores: np.ndarray,
    class_ids: np.ndarray,
    conf_threshold: float,
    iou_threshold: float,
) -> list[int]:
    mask = scores >= conf_threshold
    if not mask.any():
        return []
    idx_all = np.nonzero(mask)[0]
    b = boxes[mask].astype(np.float32)
    s = scores[mask]
    c = class_ids[mask]
    x1 = b[:, 0] - b[:, 2] / 2
    y1 = b[:, 1] - b[:, 3] / 2
    x2 = b[:, 0] + b[:, 2] / 2
    y2 = b[:, 1] + b[:, 3] / 2
    area = (x2 - x1) * (y2 - y1)
    keep: list[int] = []
    for cls in np.unique(c):
        members = np.nonzero(c == cls)[0]
        order = members[np.argsort(-s[members], kind="stable")]
        while order.size:
            i = order[0]
            keep.append(int(idx_all[i]))
            if order.size == 1:
                break
            rest = order[1:]
            w = np.maximum(0, np.minimum(x2[i], x2[rest]) - np.maximum(x1[i], x1[rest]))
            h = np.maximum(0, np.minimum(y2[i], y2[rest]) - np.maximum(y1[i], y1[rest]))
            inter = w * h
            iou = inter / (area[i] + area[rest] - inter + 1e-6)
            order = rest[iou <= iou_threshold]
    return keep


def parse_yolo_output(raw_output: np.ndarray, confidence_threshold: float, iou_threshold: float) -> np.ndarray:
    det = np.asarray(raw_output)[0].T  # [N, 84]
    boxes = det[:, :4]
    cls_scores = det[:, 4:]
    conf = cls_scores.max(axis=1)
    cls = cls_scores.argmax(axis=1)
    keep = apply_nms(boxes, conf, cls, confidence_threshold, iou_threshold)
    if not keep:
        return np.zeros((0, 6), dtype=np.float32)
    bk = boxes[keep]
    out = np.column_stack(
        [
            bk[:, 0] - bk[:, 2] / 2,
            bk[:, 1] - bk[:, 3] / 2,
            bk[:, 0] + bk[:, 2] / 2,
            bk[:, 1] + bk[:, 3] / 2,
            conf[keep],
            cls[keep],
        ]
    )
    return out.astype(np.float32)
