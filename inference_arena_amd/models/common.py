"""Building blocks shared by the two networks + BN folding + seeded init.

The torch modules in this package are the fp32 *oracles* of the HIP
pipeline (and the CPU arm's compute path).  They reproduce the public
architectures the reference exports to ONNX (src/shared/model/exporter.py:
YOLOv5nu via ultralytics :236-266, MobileNetV2 via torchvision :368-389);
neither library is available here, so the layer structure is re-declared.
"""
from __future__ import annotations

import math

import torch
from torch import nn


def autopad(k: int, p: int | None = None) -> int:
    return k // 2 if p is None else p


class ConvBNAct(nn.Module):
    """Conv2d(bias=False) -> BatchNorm2d -> activation ('silu', 'relu6', None)."""

    def __init__(self, c1: int, c2: int, k: int = 1, s: int = 1, p: int | None = None,
                 g: int = 1, act: str | None = "silu", eps: float = 1e-3):
        super().__init__()
        self.conv = nn.Conv2d(c1, c2, k, s, autopad(k, p), groups=g, bias=False)
        self.bn = nn.BatchNorm2d(c2, eps=eps)
        self.act_name = act
        self.act = {"silu": nn.SiLU(), "relu6": nn.ReLU6(), None: nn.Identity()}[act]

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.act(self.bn(self.conv(x)))


def fold_conv_bn(conv: nn.Conv2d, bn: nn.BatchNorm2d | None) -> tuple[torch.Tensor, torch.Tensor]:
    """Fold an eval-mode BatchNorm into the preceding conv: (weight, bias) fp32."""
    w = conv.weight.detach().float().cpu()
    b = conv.bias.detach().float().cpu() if conv.bias is not None else torch.zeros(w.shape[0])
    if bn is None:
        return w.clone(), b.clone()
    scale = bn.weight.detach().float().cpu() / torch.sqrt(bn.running_var.detach().float().cpu() + bn.eps)
    w = w * scale.view(-1, 1, 1, 1)
    b = (b - bn.running_mean.detach().float().cpu()) * scale + bn.bias.detach().float().cpu()
    return w, b


def fold(m: ConvBNAct) -> tuple[torch.Tensor, torch.Tensor]:
    return fold_conv_bn(m.conv, m.bn)


@torch.no_grad()
def init_random_(model: nn.Module, seed: int, alpha: float = 1.0, beta: float = 0.3) -> nn.Module:
    """Deterministic, numerically well-conditioned random init.

    Every Conv+BN weight is ``alpha * I + beta * N(0, 1/fan_in)`` where ``I``
    routes output channel o to input channel o mod Cin at the centre tap
    (identity for depthwise convs).  Plain random deep networks whose BN is
    calibrated to unit variance are chaotic: bf16 rounding noise grows ~2x
    every ~10 layers (25-40 % relative error at the YOLO head after 60 convs,
    measured against fp32).  The identity-dominant form keeps the same
    architecture, FLOPs and data-dependent outputs but behaves like a trained
    network under bf16 (~4 % head error), so GPU-vs-fp32 parity tests are
    meaningful.  Bare Conv2d/Linear layers (detect outputs, classifier) are
    N(0, 1/fan_in).
    """
    g = torch.Generator().manual_seed(int(seed))
    for mod in model.modules():
        if isinstance(mod, ConvBNAct):
            c = mod.conv
            co, ci, kh, kw = c.weight.shape
            fan_in = ci * kh * kw
            w = torch.randn(c.weight.shape, generator=g) * (beta / math.sqrt(fan_in))
            idx = torch.arange(co)
            w[idx, idx % ci if c.groups == 1 else torch.zeros_like(idx), kh // 2, kw // 2] += alpha
            c.weight.copy_(w)
            bn = mod.bn
            n = bn.num_features
            bn.weight.copy_(0.9 + 0.2 * torch.rand(n, generator=g))
            bn.bias.copy_(0.05 * torch.randn(n, generator=g))
            bn.running_mean.copy_(0.05 * torch.randn(n, generator=g))
            bn.running_var.copy_(0.9 + 0.2 * torch.rand(n, generator=g))
    for mod in model.modules():
        if isinstance(mod, (nn.Conv2d, nn.Linear)) and getattr(mod, "_arena_plain", False):
            fan_in = mod.weight[0].numel()
            mod.weight.copy_(torch.randn(mod.weight.shape, generator=g) / math.sqrt(fan_in))
            if mod.bias is not None:
                mod.bias.copy_(0.05 * torch.randn(mod.bias.shape, generator=g))
    return model


@torch.no_grad()
def calibrate_bn_(model: nn.Module, batch: torch.Tensor, seed: int, var_floor: float = 0.5) -> nn.Module:
    """Set every BN's running statistics from a calibration batch.

    One forward pass in train mode with ``momentum=None`` (cumulative average)
    records each layer's batch mean/variance given already-normalised inputs —
    what a trained network's BN statistics look like.  The affine parameters
    are then drawn around identity.  This keeps the random network's
    activations, head logits and detection counts in a realistic range.
    """
    g = torch.Generator().manual_seed(int(seed) + 7919)
    bns = [m for m in model.modules() if isinstance(m, nn.BatchNorm2d)]
    for bn in bns:
        bn.reset_running_stats()
        bn.momentum = None
        bn.weight.fill_(1.0)
        bn.bias.zero_()
    model.train()
    model(batch)
    model.eval()
    for bn in bns:
        # floor tiny variances: near-constant channels would otherwise be
        # amplified by 1/sqrt(var) and dominate rounding-noise growth
        bn.running_var.clamp_(min=float(var_floor) * float(bn.running_var.median()))
        n = bn.num_features
        bn.weight.copy_(0.8 + 0.4 * torch.rand(n, generator=g))
        bn.bias.copy_(0.1 * torch.randn(n, generator=g))
        bn.momentum = 0.1
    return model


def plain(m: nn.Module) -> nn.Module:
    """Mark a bare Conv2d/Linear for init_random_."""
    m._arena_plain = True  # type: ignore[attr-defined]
    return m
