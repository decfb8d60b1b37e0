"""Deterministic construction of the arena's two networks.

The reference exports pretrained YOLOv5nu / MobileNetV2 weights
(src/shared/model/exporter.py:192-415).  Without network access the arena
builds *random-init* networks of exactly those architectures, made
numerically realistic by calibrating every BatchNorm on synthetic images
(``calibrate_bn_``), and shifts the detector's class-logit bias so that a
useful fraction of images yields the reference workload's 3-5 detections
(the synthetic test set is then curated exactly like the reference curates
COCO: inference_arena_amd/data/curator.py).
"""
from __future__ import annotations

import functools

import numpy as np
import torch

from ..data.synthetic import synthetic_images
from ..processing.mobilenet_preprocess import MobileNetPreprocessor
from ..processing.transforms import letterbox
from .common import calibrate_bn_
from .mobilenetv2 import MobileNetV2, build_mobilenetv2
from .yolov5nu import YOLOv5nu, build_yolov5nu

# Logit shift applied to every class output of the random detector: the
# shift that maximised the share of synthetic images with 3-5 detections
# (conf 0.5, IoU 0.45) in a sweep over -40..0 (about 20 % of images).
DEFAULT_CLS_SHIFT = -28.0


def _yolo_batch(imgs, size=640) -> torch.Tensor:
    xs = [letterbox(i, size)[0].astype(np.float32).transpose(2, 0, 1) / 255.0 for i in imgs]
    return torch.from_numpy(np.stack(xs))


def _crop_batch(imgs, n: int, seed: int) -> torch.Tensor:
    rng = np.random.default_rng(seed)
    pre = MobileNetPreprocessor()
    out = []
    for k in range(n):
        im = imgs[k % len(imgs)]
        h, w = im.shape[:2]
        cw, ch = int(rng.integers(w // 8, w // 2)), int(rng.integers(h // 8, h // 2))
        x0, y0 = int(rng.integers(0, w - cw)), int(rng.integers(0, h - ch))
        out.append(pre(im[y0 : y0 + ch, x0 : x0 + cw]).tensor[0])
    return torch.from_numpy(np.stack(out))


def make_yolo(seed: int = 0, cls_shift: float = DEFAULT_CLS_SHIFT) -> YOLOv5nu:
    torch.manual_seed(seed)
    m = build_yolov5nu(seed)
    calibrate_bn_(m, _yolo_batch(synthetic_images(4, 1000 + seed)), seed)
    with torch.no_grad():
        for seq in m.detect.cv3:
            seq[2].bias += cls_shift
    return m


def make_mobilenet(seed: int = 1) -> MobileNetV2:
    torch.manual_seed(seed)
    m = build_mobilenetv2(seed)
    calibrate_bn_(m, _crop_batch(synthetic_images(4, 2000 + seed), 16, seed), seed)
    return m


@functools.lru_cache(maxsize=4)
def default_models(seed: int = 0) -> tuple[YOLOv5nu, MobileNetV2]:
    """(detector, classifier) for a weight seed; cached per process."""
    with torch.random.fork_rng():
        return make_yolo(seed), make_mobilenet(seed + 1)


def resolve_models(models_dir: str | None = None, seed: int = 0) -> tuple[YOLOv5nu, MobileNetV2]:
    """Models for a service: weights from ``models_dir`` when present — flat
    ``<dir>/<name>.safetensors`` files (monolithic/microservices init layout) or a
    repository ``<dir>/<name>/<v>/model.safetensors`` — otherwise the seeded networks.
    (Reference services verify their model files at start-up:
    architectures/monolithic/app/main.py:46-67.)"""
    from pathlib import Path

    if models_dir:
        from ..repository.store import load_module, scan_repository

        d = Path(models_dir)
        flat = [d / "yolov5n.safetensors", d / "mobilenetv2.safetensors"]
        if all(f.exists() for f in flat):
            return load_module(flat[0], "yolov5n"), load_module(flat[1], "mobilenetv2")
        if d.is_dir():
            e = scan_repository(d)
            if "yolov5n" in e and "mobilenetv2" in e:
                return (load_module(e["yolov5n"].model_file(), "yolov5n"),
                        load_module(e["mobilenetv2"].model_file(), "mobilenetv2"))
    return default_models(seed)
