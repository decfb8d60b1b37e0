"""Host NMS == a literal transcription of the reference algorithm."""
from __future__ import annotations

import numpy as np

from inference_arena_amd.postprocess import apply_nms, parse_yolo_output


def _reference_nms(boxes, scores, class_ids, conf, iou_thr):
    # literal per-class greedy loop (architectures/monolithic/app/postprocess.py:76-160)
    mask = scores >= conf
    if not mask.any():
        return []
    boxes, scores, class_ids = boxes[mask], scores[mask], class_ids[mask]
    orig = np.where(mask)[0]
    x1 = boxes[:, 0] - boxes[:, 2] / 2
    y1 = boxes[:, 1] - boxes[:, 3] / 2
    x2 = boxes[:, 0] + boxes[:, 2] / 2
    y2 = boxes[:, 1] + boxes[:, 3] / 2
    keep = []
    for cls in np.unique(class_ids):
        cm = class_ids == cls
        cx1, cy1, cx2, cy2, cs = x1[cm], y1[cm], x2[cm], y2[cm], scores[cm]
        ci = np.where(cm)[0]
        order = cs.argsort(kind="stable")[::-1]
        while len(order) > 0:
            i = order[0]
            keep.append(orig[ci[i]])
            if len(order) == 1:
                break
            xx1 = np.maximum(cx1[i], cx1[order[1:]])
            yy1 = np.maximum(cy1[i], cy1[order[1:]])
            xx2 = np.minimum(cx2[i], cx2[order[1:]])
            yy2 = np.minimum(cy2[i], cy2[order[1:]])
            inter = np.maximum(0, xx2 - xx1) * np.maximum(0, yy2 - yy1)
            a_i = (cx2[i] - cx1[i]) * (cy2[i] - cy1[i])
            a_o = (cx2[order[1:]] - cx1[order[1:]]) * (cy2[order[1:]] - cy1[order[1:]])
            iou = inter / (a_i + a_o - inter + 1e-6)
            order = order[np.where(iou <= iou_thr)[0] + 1]
    return keep


def test_nms_matches_literal_reference():
    rng = np.random.default_rng(0)
    for trial in range(20):
        n = int(rng.integers(1, 400))
        xy = rng.uniform(0, 640, (n, 2))
        wh = rng.uniform(5, 200, (n, 2))
        boxes = np.concatenate([xy, wh], 1).astype(np.float32)
        scores = rng.uniform(0, 1, n).astype(np.float32)
        cls = rng.integers(0, 5, n)
        assert apply_nms(boxes, scores, cls, 0.5, 0.45) == [int(k) for k in _reference_nms(boxes, scores, cls, 0.5, 0.45)]


def test_parse_yolo_output_format_and_order():
    out = np.zeros((1, 84, 6), np.float32)
    out[0, :4, 0] = [100, 100, 50, 50]
    out[0, 4 + 3, 0] = 0.9
    out[0, :4, 1] = [102, 101, 50, 50]  # overlaps box 0, same class, lower score -> suppressed
    out[0, 4 + 3, 1] = 0.8
    out[0, :4, 2] = [102, 101, 50, 50]  # same box, other class -> kept
    out[0, 4 + 1, 2] = 0.7
    out[0, :4, 3] = [400, 400, 20, 20]
    out[0, 4 + 3, 3] = 0.6
    out[0, 4 + 5, 4] = 0.3  # below threshold
    det = parse_yolo_output(out, 0.5, 0.45)
    assert det.shape == (3, 6) and det.dtype == np.float32
    assert det[:, 5].tolist() == [1, 3, 3]  # class asc, then score desc
    assert det[1, :4].tolist() == [75, 75, 125, 125]
    assert det[:, 4].tolist() == [np.float32(0.7), np.float32(0.9), np.float32(0.6)]


def test_parse_yolo_output_empty():
    assert parse_yolo_output(np.zeros((1, 84, 10), np.float32), 0.5, 0.45).shape == (0, 6)
