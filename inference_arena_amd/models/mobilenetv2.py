"""MobileNetV2 (torchvision layout, width 1.0, 224x224) — fp32 oracle.

The reference classifier is torchvision ``mobilenet_v2(IMAGENET1K_V1)``
exported to ONNX [1, 3, 224, 224] -> [1, 1000]
(src/shared/model/exporter.py:323-415; experiment.yaml:213-225).  Pretrained
weights cannot be fetched here; the arena uses seeded random init and can
import a torchvision state_dict when one is present locally
(``load_torchvision_state_dict``).

Shapes per layer: SURVEY.md Appendix A (52 convs + FC, 0.30 GMAC).
"""
from __future__ import annotations

import torch
from torch import nn

from .common import ConvBNAct, init_random_, plain

# (expand t, out c, repeats n, first stride s)
IR_SETTINGS = [(1, 16, 1, 1), (6, 24, 2, 2), (6, 32, 3, 2), (6, 64, 4, 2), (6, 96, 3, 1), (6, 160, 3, 2), (6, 320, 1, 1)]
NUM_CLASSES = 1000


class InvertedResidual(nn.Module):
    def __init__(self, inp: int, oup: int, stride: int, expand_ratio: int):
        super().__init__()
        hidden = inp * expand_ratio
        self.inp, self.oup, self.stride, self.hidden = inp, oup, stride, hidden
        self.use_res = stride == 1 and inp == oup
        self.expand = ConvBNAct(inp, hidden, 1, 1, act="relu6", eps=1e-5) if expand_ratio != 1 else None
        self.dw = ConvBNAct(hidden, hidden, 3, stride, g=hidden, act="relu6", eps=1e-5)
        self.project = ConvBNAct(hidden, oup, 1, 1, act=None, eps=1e-5)

    def forward(self, x):
        y = x if self.expand is None else self.expand(x)
        y = self.project(self.dw(y))
        return x + y if self.use_res else y


class MobileNetV2(nn.Module):
    def __init__(self, num_classes: int = NUM_CLASSES):
        super().__init__()
        self.stem = ConvBNAct(3, 32, 3, 2, act="relu6", eps=1e-5)
        blocks = []
        inp = 32
        for t, c, n, s in IR_SETTINGS:
            for i in range(n):
                blocks.append(InvertedResidual(inp, c, s if i == 0 else 1, t))
                inp = c
        self.blocks = nn.Sequential(*blocks)
        self.head = ConvBNAct(inp, 1280, 1, 1, act="relu6", eps=1e-5)
        self.dropout = nn.Dropout(0.2)
        self.fc = plain(nn.Linear(1280, num_classes))

    def forward(self, x):
        """[B, 3, 224, 224] ImageNet-normalised -> [B, 1000] logits."""
        x = self.head(self.blocks(self.stem(x)))
        x = torch.flatten(nn.functional.adaptive_avg_pool2d(x, 1), 1)
        return self.fc(self.dropout(x))


def build_mobilenetv2(seed: int = 1) -> MobileNetV2:
    return init_random_(MobileNetV2(), seed).eval()


def load_torchvision_state_dict(model: MobileNetV2, sd: dict[str, torch.Tensor]) -> MobileNetV2:
    """Map a torchvision mobilenet_v2 state_dict onto this module layout."""
    mine: dict[str, torch.Tensor] = {}

    def cbn(dst: str, src: str):
        mine[f"{dst}.conv.weight"] = sd[f"{src}.0.weight"]
        for k in ("weight", "bias", "running_mean", "running_var"):
            mine[f"{dst}.bn.{k}"] = sd[f"{src}.1.{k}"]

    cbn("stem", "features.0")
    for i, blk in enumerate(model.blocks):
        base = f"features.{i + 1}.conv"
        j = 0
        if blk.expand is not None:
            cbn(f"blocks.{i}.expand", f"{base}.0")
            j = 1
        cbn(f"blocks.{i}.dw", f"{base}.{j}")
        mine[f"blocks.{i}.project.conv.weight"] = sd[f"{base}.{j + 1}.weight"]
        for k in ("weight", "bias", "running_mean", "running_var"):
            mine[f"blocks.{i}.project.bn.{k}"] = sd[f"{base}.{j + 2}.{k}"]
    cbn("head", "features.18")
    mine["fc.weight"] = sd["classifier.1.weight"]
    mine["fc.bias"] = sd["classifier.1.bias"]
    model.load_state_dict(mine, strict=False)
    return model
