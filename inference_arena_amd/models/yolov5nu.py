"""YOLOv5nu (ultralytics 'yolov5n.pt' re-exported anchor-free) — fp32 oracle.

The reference's detector is the Ultralytics anchor-free YOLOv5nu: a YOLOv5
backbone/neck (Conv/C3/SPPF, depth 0.33, width 0.25) with the YOLOv8 Detect
head (DFL, reg_max 16, no objectness), exported to ONNX as
[1, 3, 640, 640] -> [1, 84, 8400] (experiment.yaml:199-207;
src/shared/data/curator.py:175-178; architectures/monolithic/app/postprocess.py:18-41).

Shapes per layer: SURVEY.md Appendix A (75 convs, 3.86 GMAC at 640).
"""
from __future__ import annotations

import torch
from torch import nn

from .common import ConvBNAct, init_random_, plain

NC = 80
REG_MAX = 16
STRIDES = (8, 16, 32)


class Bottleneck(nn.Module):
    def __init__(self, c1: int, c2: int, shortcut: bool = True):
        super().__init__()
        self.cv1 = ConvBNAct(c1, c2, 1, 1)
        self.cv2 = ConvBNAct(c2, c2, 3, 1)
        self.add = shortcut and c1 == c2

    def forward(self, x):
        y = self.cv2(self.cv1(x))
        return x + y if self.add else y


class C3(nn.Module):
    def __init__(self, c1: int, c2: int, n: int = 1, shortcut: bool = True):
        super().__init__()
        c_ = c2 // 2
        self.c_ = c_
        self.cv1 = ConvBNAct(c1, c_, 1, 1)
        self.cv2 = ConvBNAct(c1, c_, 1, 1)
        self.cv3 = ConvBNAct(2 * c_, c2, 1, 1)
        self.m = nn.Sequential(*(Bottleneck(c_, c_, shortcut) for _ in range(n)))

    def forward(self, x):
        return self.cv3(torch.cat((self.m(self.cv1(x)), self.cv2(x)), 1))


class SPPF(nn.Module):
    def __init__(self, c1: int, c2: int, k: int = 5):
        super().__init__()
        c_ = c1 // 2
        self.c_ = c_
        self.cv1 = ConvBNAct(c1, c_, 1, 1)
        self.cv2 = ConvBNAct(c_ * 4, c2, 1, 1)
        self.m = nn.MaxPool2d(k, 1, k // 2)

    def forward(self, x):
        x = self.cv1(x)
        y1 = self.m(x)
        y2 = self.m(y1)
        return self.cv2(torch.cat((x, y1, y2, self.m(y2)), 1))


def make_anchors(sizes, strides, offset: float = 0.5, device=None):
    pts, sts = [], []
    for (h, w), s in zip(sizes, strides):
        sx = torch.arange(w, dtype=torch.float32, device=device) + offset
        sy = torch.arange(h, dtype=torch.float32, device=device) + offset
        yy, xx = torch.meshgrid(sy, sx, indexing="ij")
        pts.append(torch.stack((xx, yy), -1).view(-1, 2))
        sts.append(torch.full((h * w, 1), float(s), dtype=torch.float32, device=device))
    return torch.cat(pts), torch.cat(sts)


class Detect(nn.Module):
    def __init__(self, nc: int = NC, ch: tuple[int, ...] = (64, 128, 256)):
        super().__init__()
        self.nc = nc
        self.reg_max = REG_MAX
        self.no = nc + 4 * REG_MAX
        c2 = max(16, ch[0] // 4, REG_MAX * 4)
        c3 = max(ch[0], min(nc, 100))
        self.c2, self.c3 = c2, c3
        self.cv2 = nn.ModuleList(
            nn.Sequential(ConvBNAct(x, c2, 3), ConvBNAct(c2, c2, 3), plain(nn.Conv2d(c2, 4 * REG_MAX, 1)))
            for x in ch
        )
        self.cv3 = nn.ModuleList(
            nn.Sequential(ConvBNAct(x, c3, 3), ConvBNAct(c3, c3, 3), plain(nn.Conv2d(c3, nc, 1))) for x in ch
        )
        self.register_buffer("proj", torch.arange(REG_MAX, dtype=torch.float32), persistent=False)

    def head_maps(self, feats):
        """Raw per-level head outputs [B, 64 + nc, h, w] (box logits then class logits)."""
        return [torch.cat((self.cv2[i](f), self.cv3[i](f)), 1) for i, f in enumerate(feats)]

    def decode(self, maps):
        b = maps[0].shape[0]
        sizes = [m.shape[2:] for m in maps]
        x = torch.cat([m.reshape(b, self.no, -1) for m in maps], 2)
        box, cls = x.split((4 * REG_MAX, self.nc), 1)
        a = box.shape[2]
        prob = box.view(b, 4, REG_MAX, a).transpose(2, 1).softmax(1)  # [b, 16, 4, a]
        dist = (prob * self.proj.view(1, -1, 1, 1)).sum(1)  # [b, 4, a]
        anchors, strides = make_anchors(sizes, STRIDES, device=x.device)
        anchors = anchors.t().unsqueeze(0)
        lt, rb = dist.chunk(2, 1)
        x1y1 = anchors - lt
        x2y2 = anchors + rb
        xywh = torch.cat(((x1y1 + x2y2) / 2, x2y2 - x1y1), 1) * strides.t().unsqueeze(0)
        return torch.cat((xywh, cls.sigmoid()), 1)

    def forward(self, feats):
        return self.decode(self.head_maps(feats))


class YOLOv5nu(nn.Module):
    """Backbone/neck indices follow ultralytics cfg/models/v5/yolov5.yaml (n scale)."""

    def __init__(self, nc: int = NC):
        super().__init__()
        self.b0 = ConvBNAct(3, 16, 6, 2, 2)
        self.b1 = ConvBNAct(16, 32, 3, 2)
        self.b2 = C3(32, 32, 1)
        self.b3 = ConvBNAct(32, 64, 3, 2)
        self.b4 = C3(64, 64, 2)
        self.b5 = ConvBNAct(64, 128, 3, 2)
        self.b6 = C3(128, 128, 3)
        self.b7 = ConvBNAct(128, 256, 3, 2)
        self.b8 = C3(256, 256, 1)
        self.b9 = SPPF(256, 256, 5)
        self.h10 = ConvBNAct(256, 128, 1, 1)
        self.h13 = C3(256, 128, 1, False)
        self.h14 = ConvBNAct(128, 64, 1, 1)
        self.h17 = C3(128, 64, 1, False)
        self.h18 = ConvBNAct(64, 64, 3, 2)
        self.h20 = C3(128, 128, 1, False)
        self.h21 = ConvBNAct(128, 128, 3, 2)
        self.h23 = C3(256, 256, 1, False)
        self.detect = Detect(nc, (64, 128, 256))
        self.up = nn.Upsample(scale_factor=2, mode="nearest")

    def features(self, x):
        x = self.b1(self.b0(x))
        x = self.b3(self.b2(x))
        p3b = self.b4(x)
        p4b = self.b6(self.b5(p3b))
        x = self.b9(self.b8(self.b7(p4b)))
        h10 = self.h10(x)
        x = self.h13(torch.cat((self.up(h10), p4b), 1))
        h14 = self.h14(x)
        p3 = self.h17(torch.cat((self.up(h14), p3b), 1))
        p4 = self.h20(torch.cat((self.h18(p3), h14), 1))
        p5 = self.h23(torch.cat((self.h21(p4), h10), 1))
        return [p3, p4, p5]

    def head_maps(self, x):
        return self.detect.head_maps(self.features(x))

    def forward(self, x):
        """[B, 3, 640, 640] in [0, 1] -> [B, 84, 8400] (xywh pixels + class scores)."""
        return self.detect(self.features(x))


def build_yolov5nu(seed: int = 0, cls_bias_shift: float = 0.0) -> YOLOv5nu:
    m = init_random_(YOLOv5nu(), seed).eval()
    if cls_bias_shift:
        with torch.no_grad():
            for seq in m.detect.cv3:
                seq[2].bias += cls_bias_shift
    return m
